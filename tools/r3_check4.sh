#!/bin/bash
# cfg5 binning: cap on scatter workgroups per CU (LDS floor) A/B; cfg4 training step kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=relightable3dgaussians-w_amd/lib
BENCH_ARGS="--config cfg5 --no-minibatch" STEPS=10 bash tools/variants.sh base lds64=$L/lds64/libgsr.so base lds64=$L/lds64/libgsr.so
rm -rf gpurun_out/cfg4_kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg4_kt -- python3 bench.py --config cfg4 --steps 10 \
  --warmup 3 > gpurun_out/cfg4_kt.log 2>&1
rc=$?; echo "cfg4 kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/rocpd_top.py gpurun_out/cfg4_kt 70 > gpurun_out/cfg4_top.txt; head -70 gpurun_out/cfg4_top.txt
rm -rf gpurun_out/cfg4_kt
BENCH_ARGS="--config cfg5 --no-minibatch" STEPS=10 bash tools/variants.sh lds80=$L/lds80/libgsr.so
