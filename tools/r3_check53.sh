#!/bin/bash
# round 3: the depth sort storing no keys in its last pass (lib/nk) against storing them (lib/base):
# the GPU suite on nk, then kernel traces at cfg2 and cfg5
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
L=$R/relightable3dgaussians-w_amd/lib
for v in nk; do
  cd $R && GSR_LIB_PATH=$L/$v/libgsr.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/kt53_pytest_$v.log 2>&1 \
    || { echo "pytest $v failed"; tail -30 gpurun_out/kt53_pytest_$v.log; exit 1; }
  tail -1 gpurun_out/kt53_pytest_$v.log
done
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in cfg2 cfg5; do
  steps=20; [ $cfg = cfg5 ] && steps=5
  for v in base nk base nk; do
    i=$((i+1)); d="$R/gpurun_out/kt53_${i}_${cfg}_$v"; rm -rf "$d"
    GSR_LIB_PATH=$L/$v/libgsr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$d" -- python3 "$R/bench.py" --config $cfg --steps $steps --warmup 3 --no-cpu-baseline \
      --no-refalgo --no-train --no-minibatch > "$d.log" 2>&1 || { echo "$cfg $v failed"; tail -20 "$d.log"; exit 1; }
    echo "$i $cfg $v ok"
  done
done
