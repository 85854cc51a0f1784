#!/bin/bash
# round 3: per-frame super-tile height (8x8 tiles past 682 super-tiles): the whole GPU suite,
# then cfg5 with the automatic choice against a build forced to 8x4, and cfg2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_suite.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 gpurun_out/r3_gpu_suite.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3_gpu_suite.log | head; exit $rc; }
L=relightable3dgaussians-w_amd/lib
BENCH_ARGS="--config cfg5 --no-minibatch" STEPS=10 bash tools/variants.sh auto st84=$L/st84/libgsr.so auto st84=$L/st84/libgsr.so || exit 1
STEPS=30 bash tools/variants.sh auto auto
