#!/bin/bash
# round 3: kernel times of the SSIM variants under the cfg4 iteration (rocprofv3 kernel trace)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=relightable3dgaussians-w_amd/lib
for v in ssold base ss1 ssnp; do
  lib=$PWD/$L/libgsr.so; [ $v = base ] || lib=$PWD/$L/$v/libgsr.so
  GSR_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ss_$v -o run -- \
    python bench.py --config cfg4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3_ssp_$v.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_ss_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "k_ssim" "$f" | cut -d, -f1-4
done
