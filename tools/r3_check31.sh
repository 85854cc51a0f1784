#!/bin/bash
# round 3: the epilogue backward tiled through LDS: relit tests, then the one-stream cfg4 trace
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_relit.py \
  "tests/test_gpu_fullsize.py::test_cfg3_relit_render_at_size" "tests/test_gpu_fullsize.py::test_cfg5_relit_render_fused_matches_calls" \
  tests/test_gpu_render_golden.py > gpurun_out/r3_t31.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED" gpurun_out/r3_t31.log | head; exit 1; }
echo "tests ok"; tail -1 gpurun_out/r3_t31.log
bash tools/r3_check29.sh
