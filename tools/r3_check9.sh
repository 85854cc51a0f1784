#!/bin/bash
# round 3: super-tile binning block size (GSR_ST_G) at cfg5 and cfg2, with the binning exactness test per variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=relightable3dgaussians-w_amd/lib
for g in 4096 8192; do
  GSR_LIB_PATH=$PWD/$L/g$g/libgsr.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    "tests/test_gpu_fullsize.py::test_large_frame_binning_exact" "tests/test_gpu_fullsize.py::test_cfg2_binning_invariants" tests/test_gpu_rasterizer.py > gpurun_out/r3_bin_g$g.log 2>&1 || { echo "bin test g$g failed"; tail -20 gpurun_out/r3_bin_g$g.log; exit 1; }
  echo "g$g binning tests ok"
done
BENCH_ARGS="--config cfg5 --no-minibatch" STEPS=10 bash tools/variants.sh base g2048=$L/g2048/libgsr.so g4096=$L/g4096/libgsr.so g8192=$L/g8192/libgsr.so base g4096=$L/g4096/libgsr.so || exit 1
STEPS=30 bash tools/variants.sh base g2048=$L/g2048/libgsr.so g4096=$L/g4096/libgsr.so g8192=$L/g8192/libgsr.so
