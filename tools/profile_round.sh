#!/bin/bash
# rocprofv3 evidence for bench.py: (1) kernel trace + stats, (2)/(3) separate PMC passes for
# FETCH_SIZE and WRITE_SIZE of the dominant kernel (no trace domains mixed with --pmc).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="${1:-r01}"
KREGEX="${2:-k_render_bwd}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_kt" \
  -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/prof_${TAG}_kt.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; tail -3 "$R/gpurun_out/prof_${TAG}_kt.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KREGEX" --output-format csv \
  -d "$R/gpurun_out/prof_${TAG}_fetch" -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline \
  > "$R/gpurun_out/prof_${TAG}_fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KREGEX" --output-format csv \
  -d "$R/gpurun_out/prof_${TAG}_write" -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline \
  > "$R/gpurun_out/prof_${TAG}_write.log" 2>&1
rc=$?; echo "write rc=$rc"; exit $rc
