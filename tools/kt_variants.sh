#!/bin/bash
# kernel-trace A/B: tools/kt_variants.sh "<bench args>" variant... (variant = lib/<v>/libgsr.so, "new" = lib/libgsr.so)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
ARGS="$1"; shift
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
L=$R/relightable3dgaussians-w_amd/lib
for v in "$@"; do
  lib=$L/$v/libgsr.so; [ $v = new ] && lib=$L/libgsr.so
  rm -rf "$R/gpurun_out/ktv_$v"
  GSR_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ktv_$v" \
    -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/ktv_$v.log" 2>&1 || { echo "$v failed"; exit 1; }
  echo "$v ok"
done
