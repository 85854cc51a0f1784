#!/bin/bash
# round 3: depth sort in three 9-bit passes over a range-reduced key (default) against 4 x 8 bits
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=relightable3dgaussians-w_amd/lib
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_gpu_fullsize.py::test_large_frame_binning_exact" "tests/test_gpu_fullsize.py::test_cfg2_binning_invariants" \
  "tests/test_gpu_fullsize.py::test_full_preprocess_bit_exact" tests/test_gpu_rasterizer.py tests/test_gpu_cache.py \
  > gpurun_out/r3_d9_tests.log 2>&1 || { echo "d9 tests failed"; tail -30 gpurun_out/r3_d9_tests.log; exit 1; }
echo "d9 tests ok"; tail -2 gpurun_out/r3_d9_tests.log
STEPS=30 bash tools/variants.sh base d8=$L/d8/libgsr.so base d8=$L/d8/libgsr.so || exit 1
BENCH_ARGS="--config cfg5 --no-minibatch" STEPS=10 bash tools/variants.sh base d8=$L/d8/libgsr.so
