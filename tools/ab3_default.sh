#!/bin/bash
# default-bench (3 streams) A/B: tools-free loop, one line per run
R="${GRAFT_REPO_ROOT:-/root/repo}"; L=$R/relightable3dgaussians-w_amd/lib
for v in "$@"; do
  lib=$L/$v/libgsr.so; [ $v = new ] && lib=$L/libgsr.so
  GSR_LIB_PATH=$lib timeout -k 10 200 python3 $R/bench.py --steps 30 --warmup 5 --no-relit --no-train --no-refalgo --no-cpu-baseline > $R/gpurun_out/ab3_$v.$RANDOM.log 2>&1 || exit 1
  echo "$v done"
done
