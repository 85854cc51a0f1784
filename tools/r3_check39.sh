#!/bin/bash
# round 3: culled Gaussians' record/rect/Jacobian rows written with defaults (whole lines):
# parity, then kernel traces with half the cloud culled at random (base vs new)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rasterizer.py \
  "tests/test_gpu_fullsize.py::test_full_preprocess_bit_exact" tests/test_gpu_cache.py > gpurun_out/r3_t39.log 2>&1 \
  || { echo "tests failed"; grep -E "^E |FAILED" gpurun_out/r3_t39.log | head; exit 1; }
echo "tests ok"; tail -1 gpurun_out/r3_t39.log
cd /tmp && export TMPDIR=/tmp
for v in base new base new; do
  rm -rf "$R/gpurun_out/ktc_$v"
  GSR_LIB_PATH=$R/relightable3dgaussians-w_amd/lib/$v/libgsr.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    --output-format csv -d "$R/gpurun_out/ktc_$v" -- python3 "$R/tools/culled_time.py" 0.5 20 > "$R/gpurun_out/ktc_$v.log" 2>&1 \
    || { tail -5 "$R/gpurun_out/ktc_$v.log"; exit 1; }
  echo -n "$v: "; grep "call pair" "$R/gpurun_out/ktc_$v.log"
done
