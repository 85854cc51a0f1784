#!/bin/bash
# rocprofv3 evidence for bench.py: (1) kernel trace + stats, (2)/(3) separate PMC passes for
# FETCH_SIZE and WRITE_SIZE over every kernel (no trace domains mixed with --pmc), then
# tools/profile_summary.py writes profiles/<tag>_{kernel_stats.csv,hbm_traffic.json,summary.md}.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="${1:-r01}"
shift || true
EXTRA="$*"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
rm -rf "$R/gpurun_out/prof_${TAG}_kt" "$R/gpurun_out/prof_${TAG}_fetch" "$R/gpurun_out/prof_${TAG}_write" \
  "$R/gpurun_out/prof_${TAG}_valu"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_kt" \
  -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-refalgo --no-relit --no-train --no-minibatch --no-clustered --streams 1 $EXTRA > "$R/gpurun_out/prof_${TAG}_kt.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; grep '^{"metric"' "$R/gpurun_out/prof_${TAG}_kt.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv \
  -d "$R/gpurun_out/prof_${TAG}_fetch" -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-refalgo --no-relit --no-train --no-minibatch --no-clustered --streams 1 $EXTRA \
  > "$R/gpurun_out/prof_${TAG}_fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv \
  -d "$R/gpurun_out/prof_${TAG}_write" -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-refalgo --no-relit --no-train --no-minibatch --no-clustered --streams 1 $EXTRA \
  > "$R/gpurun_out/prof_${TAG}_write.log" 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv \
  -d "$R/gpurun_out/prof_${TAG}_valu" -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-refalgo --no-relit --no-train --no-minibatch --no-clustered --streams 1 $EXTRA \
  > "$R/gpurun_out/prof_${TAG}_valu.log" 2>&1
rc=$?; echo "valu rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 "$R/tools/profile_summary.py" "$TAG"
