#!/bin/bash
# round 3: as r3_check45.sh, the rects packed on their way into LDS (pass 0), kernel traces only
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
L=$R/relightable3dgaussians-w_amd/lib
cd $R
cd /tmp && export TMPDIR=/tmp
mkdir -p $L/base && cp $L/libgsr.so $L/base/
i=0
for cfg in cfg2 cfg5; do
  steps=20; [ $cfg = cfg5 ] && steps=5
  for v in base pk base pk; do
    i=$((i+1)); d="$R/gpurun_out/kt46_${i}_${cfg}_$v"; rm -rf "$d"
    GSR_LIB_PATH=$L/$v/libgsr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$d" -- python3 "$R/bench.py" --config $cfg --steps $steps --warmup 3 --no-cpu-baseline \
      --no-refalgo --no-train --no-minibatch > "$d.log" 2>&1 || { echo "$cfg $v failed"; tail -20 "$d.log"; exit 1; }
    echo "$i $cfg $v ok"
  done
done
