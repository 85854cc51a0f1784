#!/bin/bash
# round 3: each 64-B relit feature row written whole by one kernel (the shade writes the
# foreground rows, k_relit_prep the sky rows): relit/train tests, then the one-stream trace
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py tests/test_gpu_relit.py \
  tests/test_gpu_render_golden.py tests/test_gpu_train.py tests/test_gpu_channels.py \
  "tests/test_gpu_fullsize.py::test_cfg3_relit_render_at_size" > gpurun_out/r3_t38.log 2>&1 \
  || { echo "tests failed"; grep -E "^E |FAILED" gpurun_out/r3_t38.log | head; exit 1; }
echo "tests ok"; tail -1 gpurun_out/r3_t38.log
bash tools/r3_check29.sh
