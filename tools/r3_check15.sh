#!/bin/bash
# round 3: relit/channels/train GPU tests + cfg4 rate + glue table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_channels.py \
  tests/test_gpu_relit.py tests/test_gpu_render_golden.py tests/test_gpu_ssim.py tests/test_gpu_trainaux.py \
  tests/test_gpu_train.py > gpurun_out/r3_t15.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r3_t15.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r3_t15.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --config cfg4 --steps 20 --warmup 5 > gpurun_out/r3_cfg4b.log 2>&1
rc=$?; echo "cfg4 rc=$rc"; tail -1 gpurun_out/r3_cfg4b.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/train_glue.py 1363637 60 > gpurun_out/train_glue5.log 2>&1; echo "glue rc=$?"
