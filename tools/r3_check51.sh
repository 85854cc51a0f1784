#!/bin/bash
# round 3: k_st_hist with one LDS histogram per block (lib/hs1) against one per wave, summed
# (lib/hs0, GSR_ST_HIST_SHARED=0): binning + rasterizer GPU tests on hs1, then
# alternating kernel traces at cfg2 and cfg5
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
L=$R/relightable3dgaussians-w_amd/lib
cd $R && GSR_LIB_PATH=$L/hs1/libgsr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py \
  tests/test_gpu_rasterizer.py tests/test_gpu_cache.py tests/test_gpu_channels.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/kt51_pytest_hs1.log 2>&1 || { echo "pytest hs1 failed"; tail -30 gpurun_out/kt51_pytest_hs1.log; exit 1; }
tail -2 gpurun_out/kt51_pytest_hs1.log
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in cfg2 cfg5; do
  steps=20; [ $cfg = cfg5 ] && steps=5
  for v in hs0 hs1 hs0 hs1; do
    i=$((i+1)); d="$R/gpurun_out/kt51_${i}_${cfg}_$v"; rm -rf "$d"
    GSR_LIB_PATH=$L/$v/libgsr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$d" -- python3 "$R/bench.py" --config $cfg --steps $steps --warmup 3 --no-cpu-baseline \
      --no-refalgo --no-train --no-minibatch > "$d.log" 2>&1 || { echo "$cfg $v failed"; tail -20 "$d.log"; exit 1; }
    echo "$i $cfg $v ok"
  done
done
