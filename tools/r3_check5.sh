#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=relightable3dgaussians-w_amd/lib
STEPS=30 bash tools/variants.sh base lean=$L/lean/libgsr.so base lean=$L/lean/libgsr.so base lean=$L/lean/libgsr.so
timeout -k 10 400 python tools/train_glue.py 1363637 60 > gpurun_out/train_glue.log 2>&1; echo "glue rc=$?"
