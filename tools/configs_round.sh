#!/bin/bash
# The secondary bench configurations (cfg3 fused render(), cfg4 training, cfg5 4K stress,
# cfg5-relit) into gpurun_out/<tag>_<cfg>.log, each under its own time limit.
set -o pipefail
TAG=${1:-r08}
mkdir -p gpurun_out
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/${TAG}_$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; grep -o '"value": [0-9.]*, "unit": "[^"]*"' gpurun_out/${TAG}_$n.log | head -1
  return $rc
}
run cfg3 --config cfg3 --steps 20 --warmup 5 && run cfg4 --config cfg4 --steps 30 --warmup 5 &&
  run cfg5 --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline --no-refalgo &&
  run cfg5r --config cfg5-relit --steps 5 --warmup 2
