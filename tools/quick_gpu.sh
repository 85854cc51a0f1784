#!/bin/bash
# One gpurun call: GPU tests (optional), bench line, kernel-trace stats of the bench.
#   tools/quick_gpu.sh [tests|notests] [extra bench args...]
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mode=${1:-tests}; shift || true
mkdir -p gpurun_out
rm -rf gpurun_out/qk
if [ "$mode" = tests ]; then
  timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
fi
timeout -k 10 200 python bench.py --no-cpu-baseline --no-refalgo --no-train "$@" > gpurun_out/b.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/qk -- python3 bench.py --steps 10 --warmup 3 --no-refalgo \
  --no-cpu-baseline --no-refalgo --no-train "$@" > gpurun_out/p.log 2>&1
python3 tools/rocpd_top.py gpurun_out/qk 60 > gpurun_out/qk_top.txt
rm -rf gpurun_out/qk
