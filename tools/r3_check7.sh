#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_relit.py \
  tests/test_gpu_render_golden.py tests/test_gpu_train.py > gpurun_out/r3_relit_tests.log 2>&1
rc=$?; echo "relit tests rc=$rc"; tail -3 gpurun_out/r3_relit_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/train_glue.py 1363637 60 > gpurun_out/train_glue2.log 2>&1; echo "glue rc=$?"
bash tools/r3_check6.sh
