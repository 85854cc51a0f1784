#!/bin/bash
# round 3: is the super-tile scatter bound by its scattered entry stores?  (timing experiments:
# stw1 = each lane's entries at consecutive slots, stw2 = no entry stores; both wrong output)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=relightable3dgaussians-w_amd/lib
for v in ${VARIANTS:-base stw1 stw2}; do
  lib=$PWD/$L/libgsr.so; [ $v = base ] || lib=$PWD/$L/$v/libgsr.so
  GSR_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stw_$v -o run -- \
    python bench.py --config cfg5 --no-cpu-baseline --no-refalgo --no-train --no-minibatch --steps 10 --warmup 3 \
    > gpurun_out/stw_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/stw_$v.log; exit 1; }
  f=$(find gpurun_out/prof_stw_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "st_scatter|st_hist|radix_scatter|render_fwd|fillBuffer" "$f" | cut -d, -f1-4
done
