#!/bin/bash
# round 3: the shade slabs stored value-major (coalesced k_shade_base_reduce): shade, relit and
# training tests, then the one-stream cfg4 trace
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_relit.py \
  tests/test_gpu_render_golden.py tests/test_gpu_train.py > gpurun_out/r3_t37.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED" gpurun_out/r3_t37.log | head; exit 1; }
echo "tests ok"; tail -1 gpurun_out/r3_t37.log
bash tools/r3_check29.sh
