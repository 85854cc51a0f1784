#!/bin/bash
# round 3: the image gradient's L1 term made in the SSIM backward: training tests, then the
# one-stream cfg4 kernel trace and the cfg4 bench
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ssim.py tests/test_gpu_train.py \
  tests/test_gpu_trainaux.py > gpurun_out/r3_t32.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED" gpurun_out/r3_t32.log | head; exit 1; }
echo "tests ok"; tail -1 gpurun_out/r3_t32.log
bash tools/r3_check29.sh || exit 1
cd "$R"
timeout -k 10 300 python bench.py --config cfg4 --steps 30 --warmup 5 > gpurun_out/r3_c4_32.log 2>&1 || exit 1
grep -o '"value": [0-9.]*, "unit": "[^"]*", "n_gpus": [0-9]*, "ranks_joined": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/r3_c4_32.log
