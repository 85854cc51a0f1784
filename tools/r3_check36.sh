#!/bin/bash
# round 3: depth-sort tile size (GSR_SORT_ITEMS keys per thread: 8 = 2048-key tiles, 12, 16) at
# cfg5 and cfg2: binning exactness, then A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=relightable3dgaussians-w_amd/lib
for v in si12 si16; do
  GSR_LIB_PATH=$PWD/$L/$v/libgsr.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    "tests/test_gpu_fullsize.py::test_large_frame_binning_exact" tests/test_gpu_rasterizer.py > gpurun_out/r3_${v}_tests.log 2>&1 \
    || { echo "$v tests failed"; grep -E "^E |FAILED" gpurun_out/r3_${v}_tests.log | head; exit 1; }
  echo "$v tests ok"
done
BENCH_ARGS="--config cfg5 --no-minibatch" STEPS=10 bash tools/variants.sh base si12=$L/si12/libgsr.so si16=$L/si16/libgsr.so base si12=$L/si12/libgsr.so si16=$L/si16/libgsr.so || exit 1
STEPS=30 bash tools/variants.sh base si12=$L/si12/libgsr.so si16=$L/si16/libgsr.so
