#!/bin/bash
# round 3: render_bwd at 5 waves per SIMD (lib/bw5) against the in-tree 4, alternating, each
# run's trace in its own directory
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/relightable3dgaussians-w_amd/lib/base && cp $R/relightable3dgaussians-w_amd/lib/libgsr.so $R/relightable3dgaussians-w_amd/lib/base/
i=0
for v in base bw5 base bw5 base bw5; do
  i=$((i+1)); d="$R/gpurun_out/kt44_${i}_$v"; rm -rf "$d"
  GSR_LIB_PATH=$R/relightable3dgaussians-w_amd/lib/$v/libgsr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d "$d" -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-refalgo --no-train \
    --no-minibatch > "$d.log" 2>&1 || { echo "$v failed"; exit 1; }
  echo "$i $v ok"
done
