#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/diag_large.py > gpurun_out/r3_diag.log 2>&1; echo "diag rc=$?"
bash tools/ab_r3.sh 2>&1 | tee gpurun_out/r3_ab.log
