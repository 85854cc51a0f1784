#!/bin/bash
# round 3: the fused training bookkeeping kernels (gsr_trainaux.hip) -- parity tests, the
# training tests, the glue profile and the cfg4 training iteration rate
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_trainaux.py \
  tests/test_gpu_train.py > gpurun_out/r3_trainaux_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -25 gpurun_out/r3_trainaux_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/train_glue.py 1363637 60 > gpurun_out/train_glue3.log 2>&1; echo "glue rc=$?"
[ $? -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --config cfg4 --steps 20 --warmup 5 > gpurun_out/r3_cfg4.log 2>&1
rc=$?; echo "cfg4 rc=$rc"; tail -2 gpurun_out/r3_cfg4.log
