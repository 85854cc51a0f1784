#!/bin/bash
# round 3: the backward's ninth sum as four row partials to four slots of the accumulator line
# lib/s8s): parity, then cfg2 kernel trace A/B
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
L=relightable3dgaussians-w_amd/lib
GSR_LIB_PATH=$R/$L/s8s/libgsr.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_rasterizer.py tests/test_gpu_det.py "tests/test_gpu_fullsize.py::test_full_sampled_tiles_backward" \
  > gpurun_out/r3_s8s_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED" gpurun_out/r3_s8s_tests.log | head; exit 1; }
echo "tests ok"; tail -1 gpurun_out/r3_s8s_tests.log
bash tools/kt_variants.sh '--steps 20 --warmup 5 --no-cpu-baseline --no-refalgo --no-train --no-minibatch' base s8s base s8s || exit 1
