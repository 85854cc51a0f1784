#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=relightable3dgaussians-w_amd/lib
for v in ssold base ss1 ssnp ssold base ss1 ssnp; do
  lib=$PWD/$L/libgsr.so; [ $v = base ] || lib=$PWD/$L/$v/libgsr.so
  echo "$v $(GSR_LIB_PATH=$lib timeout -k 10 120 python tools/bench_ssim.py 2>&1 | tail -1)" || exit 1
done
