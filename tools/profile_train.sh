#!/bin/bash
# rocprofv3 evidence for the cfg4 training iteration (bench.py's `train` leg, run on one stream
# by tools/train_kernels.py so kernel durations are not inflated by the two-stream overlap):
# (1) kernel trace + stats, (2)/(3)/(4) separate PMC passes FETCH_SIZE, WRITE_SIZE and
# SQ_INSTS_VALU/SALU/WAVES (counters never mixed with trace domains), then
# tools/profile_summary.py writes profiles/<tag>_{kernel_stats.csv,hbm_traffic.json,summary.md}.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="${1:-r4_cfg4}"
ITERS="${2:-10}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
for s in kt fetch write valu; do rm -rf "$R/gpurun_out/prof_${TAG}_$s"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_kt" \
  -- python3 "$R/tools/train_kernels.py" "$ITERS" > "$R/gpurun_out/prof_${TAG}_kt.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; tail -2 "$R/gpurun_out/prof_${TAG}_kt.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/prof_${TAG}_fetch" \
  -- python3 "$R/tools/train_kernels.py" 2 > "$R/gpurun_out/prof_${TAG}_fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/prof_${TAG}_write" \
  -- python3 "$R/tools/train_kernels.py" 2 > "$R/gpurun_out/prof_${TAG}_write.log" 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv \
  -d "$R/gpurun_out/prof_${TAG}_valu" -- python3 "$R/tools/train_kernels.py" 2 \
  > "$R/gpurun_out/prof_${TAG}_valu.log" 2>&1
rc=$?; echo "valu rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 "$R/tools/profile_summary.py" "$TAG" "cfg4 training iteration (tools/train_kernels.py: 1.36M fg + 0.14M sky Gaussians, 1920x1080, 4 views, one stream)"
