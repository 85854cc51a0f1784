#!/bin/bash
# Kernel-trace A/B of libgsr builds (the round-by-round A/B tool; round 3's one-off
# tools/r3_check*.sh scripts were folded into it and removed in round 4 -- git history keeps them):
#
#   tools/kt_variants.sh "<bench args>" variant...
#
# variant = lib/<v>/libgsr.so ("new" = lib/libgsr.so, the in-tree build); a variant may repeat
# (e.g. "new v5 new v5 new v5" alternates runs), each run traced into gpurun_out/ktv_<v>_<i>.
# Then: python3 tools/kt_compare.py <variant>... averages each variant's runs side by side.
# Env TOOL=train runs tools/train_kernels.py instead of bench.py (ARGS = its iteration count);
# KTP=<prefix> prefixes the run directories (ktv_<prefix><v>_<i>; kt_compare.py reads KTP too).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
ARGS="$1"; shift
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
L=$R/relightable3dgaussians-w_amd/lib
PROG="$R/bench.py"; [ "${TOOL:-bench}" = train ] && PROG="$R/tools/train_kernels.py"
i=0
for v in "$@"; do
  i=$((i+1))
  lib=$L/$v/libgsr.so; [ $v = new ] && lib=$L/libgsr.so
  [ -f "$lib" ] || { echo "no $lib"; exit 1; }
  d="$R/gpurun_out/ktv_${KTP:-}${v}_$i"; rm -rf "$d"
  GSR_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" \
    -- python3 "$PROG" $ARGS > "$d.log" 2>&1 || { echo "$v ($i) failed"; tail -5 "$d.log"; exit 1; }
  echo "$i $v ok"
done
