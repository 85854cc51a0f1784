#!/bin/bash
# round 3: 64-B accumulator lines (GSR_ACC_STRIDE=16, lib/a16): parity, cfg2 A/B, and the
# render/preprocess backward's HBM traffic (FETCH_SIZE, WRITE_SIZE passes) for both layouts
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
L=relightable3dgaussians-w_amd/lib
GSR_LIB_PATH=$R/$L/a16/libgsr.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_rasterizer.py tests/test_gpu_channels.py tests/test_gpu_det.py \
  > gpurun_out/r3_a16_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED" gpurun_out/r3_a16_tests.log | head; exit 1; }
echo "tests ok"; tail -1 gpurun_out/r3_a16_tests.log
STEPS=30 bash tools/variants.sh base a16=$L/a16/libgsr.so base a16=$L/a16/libgsr.so || exit 1
cd /tmp && export TMPDIR=/tmp
for v in base a16; do
  lib=$R/$L/libgsr.so; [ $v = a16 ] && lib=$R/$L/a16/libgsr.so
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf "$R/gpurun_out/pmc26_${v}_$c"
    GSR_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --pmc $c --kernel-include-regex "k_render_bwd|k_preprocess_bwd|k_digit_scan" \
      --output-format csv -d "$R/gpurun_out/pmc26_${v}_$c" -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline \
      --no-refalgo --no-train --no-minibatch > "$R/gpurun_out/pmc26_${v}_$c.log" 2>&1 || { echo "pmc $v $c failed"; exit 1; }
    echo "pmc $v $c ok"
  done
done
