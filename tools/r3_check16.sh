#!/bin/bash
# round 3: SSIM strip kernels (4 chunks of 32 rows per workgroup, next chunk prefetched) vs
# the single-tile kernels: SSIM tests per variant, then cfg4 iteration time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=relightable3dgaussians-w_amd/lib
for v in base ssnp ss1; do
  lib=$PWD/$L/libgsr.so; [ $v = base ] || lib=$PWD/$L/$v/libgsr.so
  GSR_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ssim.py \
    > gpurun_out/r3_ss_$v.log 2>&1 || { echo "ssim tests $v failed"; grep -E "^E |FAILED" gpurun_out/r3_ss_$v.log | head; exit 1; }
done
echo "ssim tests ok"
for v in ssold base ssnp ss1 ssold base; do
  lib=$PWD/$L/libgsr.so; [ $v = base ] || lib=$PWD/$L/$v/libgsr.so
  GSR_LIB_PATH=$lib timeout -k 10 300 python bench.py --config cfg4 --steps 20 --warmup 5 > gpurun_out/r3_ssb_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r3_ssb_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
