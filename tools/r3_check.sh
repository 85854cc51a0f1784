#!/bin/bash
# Round-3 GPU check: the half-exec VALU micro, new/changed GPU tests, the cfg3 relight bench,
# the N=2 launcher rehearsed with gloo (two ranks sharing the one GPU), and the cfg5 rocprofv3
# passes.  Each GPU step has its own limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cache.py \
  tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_render_golden.py \
  -k "large or cfg3 or cfg5_relit or full_size_step" \
  > gpurun_out/r3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config cfg3 --steps 10 --warmup 3 > gpurun_out/r3_cfg3.log 2>&1
rc=$?; echo "cfg3 rc=$rc"; tail -2 gpurun_out/r3_cfg3.log; [ $rc -eq 0 ] || exit $rc
GSR_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/r3_n2.log 2>&1
rc=$?; echo "n2 rc=$rc"; tail -3 gpurun_out/r3_n2.log; [ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh r3b_cfg5 --config cfg5 || exit $?
