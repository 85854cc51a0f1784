#!/bin/bash
# round 3: kernel trace of the depth sort, 9-bit range-reduced (default) vs 4 x 8 bits, cfg2 and cfg5
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
L=$R/relightable3dgaussians-w_amd/lib
for cfg in cfg2 cfg5; do
  for v in d9 d8; do
    lib=$L/libgsr.so; [ $v = d8 ] && lib=$L/d8/libgsr.so
    rm -rf "$R/gpurun_out/kt_${v}_${cfg}"
    GSR_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_${v}_${cfg}" \
      -- python3 "$R/bench.py" --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-refalgo --no-train --no-minibatch \
      > "$R/gpurun_out/kt_${v}_${cfg}.log" 2>&1 || { echo "$v $cfg failed"; exit 1; }
    echo "$v $cfg ok"
  done
done
