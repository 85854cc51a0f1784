#!/bin/bash
# round 3: 9-bit depth sort with the zero-fill in all four scans; A/B against 4 x 8 bits
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=relightable3dgaussians-w_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rasterizer.py \
  > gpurun_out/r3_d9b_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r3_d9b_tests.log; exit 1; }
echo "tests ok"; tail -1 gpurun_out/r3_d9b_tests.log
STEPS=30 bash tools/variants.sh base d8=$L/d8/libgsr.so base d8=$L/d8/libgsr.so base d8=$L/d8/libgsr.so || exit 1
BENCH_ARGS="--config cfg5 --no-minibatch" STEPS=10 bash tools/variants.sh base d8=$L/d8/libgsr.so base d8=$L/d8/libgsr.so
