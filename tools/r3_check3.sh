#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/diag_large2.py > gpurun_out/r3_diag2.log 2>&1; echo "diag2 rc=$?"; tail -5 gpurun_out/r3_diag2.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py \
  tests/test_gpu_rasterizer.py -k "binning or speculative or forward_parity or cfg2 or cfg5" > gpurun_out/r3_bin_tests.log 2>&1
rc=$?; echo "binning tests rc=$rc"; tail -3 gpurun_out/r3_bin_tests.log; [ $rc -eq 0 ] || exit $rc
L=relightable3dgaussians-w_amd/lib
BENCH_ARGS="--config cfg5 --no-minibatch" STEPS=10 bash tools/variants.sh stold=$L/stold/libgsr.so flat stold=$L/stold/libgsr.so flat
STEPS=30 bash tools/variants.sh stold=$L/stold/libgsr.so flat stold=$L/stold/libgsr.so flat
