#!/bin/bash
# round 3: fused view objective + unbound per-view rows: loss/train tests, cfg4 rate, glue table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ssim.py \
  tests/test_gpu_trainaux.py tests/test_gpu_train.py > gpurun_out/r3_obj_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r3_obj_tests.log | tail -5; [ $rc -eq 0 ] || { tail -40 gpurun_out/r3_obj_tests.log; exit $rc; }
timeout -k 10 400 python bench.py --config cfg4 --steps 20 --warmup 5 > gpurun_out/r3_cfg4b.log 2>&1
rc=$?; echo "cfg4 rc=$rc"; tail -1 gpurun_out/r3_cfg4b.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/train_glue.py 1363637 60 > gpurun_out/train_glue5.log 2>&1; echo "glue rc=$?"
