#!/bin/bash
# round 3: depth sort in 3 passes of 11 + 11 + 10 bits (GSR_DEPTH_BITS=11) against 4 x 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=relightable3dgaussians-w_amd/lib
GSR_LIB_PATH=$PWD/$L/d11/libgsr.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_gpu_fullsize.py::test_large_frame_binning_exact" "tests/test_gpu_fullsize.py::test_cfg2_binning_invariants" \
  tests/test_gpu_rasterizer.py > gpurun_out/r3_d11_tests.log 2>&1 || { echo "d11 tests failed"; tail -30 gpurun_out/r3_d11_tests.log; exit 1; }
echo "d11 tests ok"
STEPS=30 bash tools/variants.sh base d11=$L/d11/libgsr.so base d11=$L/d11/libgsr.so || exit 1
BENCH_ARGS="--config cfg5 --no-minibatch" STEPS=10 bash tools/variants.sh base d11=$L/d11/libgsr.so
