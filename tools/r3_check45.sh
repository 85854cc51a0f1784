#!/bin/bash
# round 3: depth-sorted rects packed to 4 bytes (lib/pk) against the in-tree 8-byte rects:
# the GPU suite on lib/pk, then alternating kernel traces at cfg2 and cfg5
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
L=$R/relightable3dgaussians-w_amd/lib
cd $R && GSR_LIB_PATH=$L/pk/libgsr.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/kt45_pytest_pk.log 2>&1 || { echo "pytest pk failed"; tail -30 gpurun_out/kt45_pytest_pk.log; exit 1; }
tail -2 gpurun_out/kt45_pytest_pk.log
cd /tmp && export TMPDIR=/tmp
mkdir -p $L/base && cp $L/libgsr.so $L/base/
i=0
for cfg in cfg2 cfg5; do
  steps=20; [ $cfg = cfg5 ] && steps=5
  for v in base pk base pk; do
    i=$((i+1)); d="$R/gpurun_out/kt45_${i}_${cfg}_$v"; rm -rf "$d"
    GSR_LIB_PATH=$L/$v/libgsr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$d" -- python3 "$R/bench.py" --config $cfg --steps $steps --warmup 3 --no-cpu-baseline \
      --no-refalgo --no-train --no-minibatch > "$d.log" 2>&1 || { echo "$cfg $v failed"; tail -20 "$d.log"; exit 1; }
    echo "$i $cfg $v ok"
  done
done
