#!/bin/bash
# Default-bench A/B (3 HIP streams, views overlapping -- the headline's mode): alternating runs of
# libgsr builds, one bench line each into gpurun_out/ab3_<variant>.<n>.log.
#   tools/ab3_default.sh variant...      (variant = lib/<v>/libgsr.so, "new" = lib/libgsr.so)
# Env AB3_ARGS adds bench arguments (e.g. "--config cfg5 --steps 10 --warmup 3").
R="${GRAFT_REPO_ROOT:-/root/repo}"; L=$R/relightable3dgaussians-w_amd/lib
for v in "$@"; do
  lib=$L/$v/libgsr.so; [ $v = new ] && lib=$L/libgsr.so
  GSR_LIB_PATH=$lib timeout -k 10 200 python3 $R/bench.py --steps 30 --warmup 5 --no-relit --no-train --no-refalgo --no-cpu-baseline ${AB3_ARGS:-} > $R/gpurun_out/ab3_$v.$RANDOM.log 2>&1 || exit 1
  echo "$v done"
done
