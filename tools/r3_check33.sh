#!/bin/bash
# round 3: cfg4 iterations/s against the number of HIP streams the views alternate over
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do for ns in 2 3 4 1; do
  timeout -k 10 300 python bench.py --config cfg4 --steps 30 --warmup 5 --streams $ns > gpurun_out/r3_c4_s$ns.log 2>&1 || exit 1
  echo -n "streams $ns: "; grep -o '"value": [0-9.]*' gpurun_out/r3_c4_s$ns.log | head -1
done; done
