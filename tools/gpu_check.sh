#!/bin/bash
# One gpurun call: the GPU suite (optionally a subset), the default bench line and a clean
# single-call kernel timeline (tools/timeline.py).  Every GPU step has its own time limit and
# the chain stops at the first failure.
#   tools/gpu_check.sh [pytest selection...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
sel="${*:-tests}"
timeout -k 10 700 python -u -m pytest $sel -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/b.log 2>&1
rc=$?; tail -1 gpurun_out/b.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
rm -rf gpurun_out/tl
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -- python3 bench.py --steps 10 --warmup 3 \
  --no-minibatch --no-refalgo --no-cpu-baseline --no-train > gpurun_out/tl.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python3 tools/timeline.py gpurun_out/tl > gpurun_out/timeline.txt; cat gpurun_out/timeline.txt
