#!/bin/bash
# round 3: preprocess / preprocess-backward / SSIM TUs without SLP packing (lib/pbns): parity
# tests, then cfg2 A/B and the SSIM kernel timing against the in-tree build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=relightable3dgaussians-w_amd/lib
GSR_LIB_PATH=$PWD/$L/pbns/libgsr.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_rasterizer.py "tests/test_gpu_fullsize.py::test_full_preprocess_bit_exact" \
  "tests/test_gpu_fullsize.py::test_full_sampled_tiles_backward" tests/test_gpu_ssim.py \
  > gpurun_out/r3_pbns_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED" gpurun_out/r3_pbns_tests.log | head; tail -3 gpurun_out/r3_pbns_tests.log; exit 1; }
echo "tests ok"; tail -1 gpurun_out/r3_pbns_tests.log
STEPS=30 bash tools/variants.sh base pbns=$L/pbns/libgsr.so base pbns=$L/pbns/libgsr.so || exit 1
for v in base pbns; do lib=$PWD/$L/libgsr.so; [ $v = pbns ] && lib=$PWD/$L/pbns/libgsr.so
  echo -n "$v "; GSR_LIB_PATH=$lib timeout -k 10 120 python tools/bench_ssim.py 2>&1 | grep k_ssim || exit 1; done
