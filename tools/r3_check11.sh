#!/bin/bash
# round 3: 8x8-tile super-tiles (GSR_ST_H=8) against 8x4: binning/rasterizer parity with the
# variant, then cfg5 and cfg2 timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=relightable3dgaussians-w_amd/lib
GSR_LIB_PATH=$PWD/$L/st88/libgsr.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_gpu_fullsize.py::test_large_frame_binning_exact" "tests/test_gpu_fullsize.py::test_cfg2_binning_invariants" \
  tests/test_gpu_rasterizer.py tests/test_gpu_channels.py > gpurun_out/r3_st88_tests.log 2>&1 || { echo "st88 tests failed"; tail -30 gpurun_out/r3_st88_tests.log; exit 1; }
echo "st88 tests ok"; tail -1 gpurun_out/r3_st88_tests.log
BENCH_ARGS="--config cfg5 --no-minibatch" STEPS=10 bash tools/variants.sh base st88=$L/st88/libgsr.so base st88=$L/st88/libgsr.so || exit 1
STEPS=30 bash tools/variants.sh base st88=$L/st88/libgsr.so base st88=$L/st88/libgsr.so
