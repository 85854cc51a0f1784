#!/bin/bash
# round 3 evidence, part 1: the whole GPU suite, smoke(), the default bench line
set -o pipefail
TAG=${1:-r3z}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/${TAG}_pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{"metric"' gpurun_out/${TAG}_bench.log | cut -c1-300
