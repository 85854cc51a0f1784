#!/bin/bash
# round 3: the 14-channel tile passes at forced occupancy (mcb4: backward 4 waves per SIMD,
# mcf5: forward 5, with spills): channel parity, then one-stream cfg4 traces
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
for v in mcb4 mcf5; do
  GSR_LIB_PATH=$R/relightable3dgaussians-w_amd/lib/$v/libgsr.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_channels.py > gpurun_out/r3_${v}_tests.log 2>&1 \
    || { echo "$v tests failed"; grep -E "^E |FAILED" gpurun_out/r3_${v}_tests.log | head; exit 1; }
  echo "$v tests ok"
done
bash tools/kt_train_variants.sh base mcb4 mcf5 base
