#!/bin/bash
# round 3: binning blocks of 512 / 2048 Gaussians (GSR_ST_G; lib/g512, lib/g2048) against 1024
# (lib/base), now that the scatter counts its own waves' entries: kernel traces at cfg2 and cfg5
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
L=$R/relightable3dgaussians-w_amd/lib
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in cfg2 cfg5; do
  steps=20; [ $cfg = cfg5 ] && steps=5
  for v in base g512 g2048 base g512 g2048; do
    i=$((i+1)); d="$R/gpurun_out/kt48_${i}_${cfg}_$v"; rm -rf "$d"
    GSR_LIB_PATH=$L/$v/libgsr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$d" -- python3 "$R/bench.py" --config $cfg --steps $steps --warmup 3 --no-cpu-baseline \
      --no-refalgo --no-train --no-minibatch > "$d.log" 2>&1 || { echo "$cfg $v failed"; tail -20 "$d.log"; exit 1; }
    echo "$i $cfg $v ok"
  done
done
