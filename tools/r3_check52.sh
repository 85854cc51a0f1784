#!/bin/bash
# round 3: the backward tile pass splitting its 64 / 128 lightest tiles per band into quadrant
# units (GSR_BWD_TAIL; lib/bt64, lib/bt128) against none (lib/base), re-measured at five waves per
# SIMD: rasterizer GPU tests on both, then kernel traces at cfg2 and cfg5
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
L=$R/relightable3dgaussians-w_amd/lib
for v in bt64 bt128; do
  cd $R && GSR_LIB_PATH=$L/$v/libgsr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_rasterizer.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/kt52_pytest_$v.log 2>&1 \
    || { echo "pytest $v failed"; tail -30 gpurun_out/kt52_pytest_$v.log; exit 1; }
  tail -1 gpurun_out/kt52_pytest_$v.log
done
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in cfg2 cfg5; do
  steps=20; [ $cfg = cfg5 ] && steps=5
  for v in base bt64 bt128 base bt64 bt128; do
    i=$((i+1)); d="$R/gpurun_out/kt52_${i}_${cfg}_$v"; rm -rf "$d"
    GSR_LIB_PATH=$L/$v/libgsr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$d" -- python3 "$R/bench.py" --config $cfg --steps $steps --warmup 3 --no-cpu-baseline \
      --no-refalgo --no-train --no-minibatch > "$d.log" 2>&1 || { echo "$cfg $v failed"; tail -20 "$d.log"; exit 1; }
    echo "$i $cfg $v ok"
  done
done
