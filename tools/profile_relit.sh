#!/bin/bash
# rocprofv3 evidence for the relit legs (BASELINE configs[2] / [4]: cfg3, cfg5-relit), one stream:
#   tools/profile_relit.sh TAG cfg3|cfg5-relit
# (1) kernel trace + stats, (2)-(4) separate PMC passes FETCH_SIZE, WRITE_SIZE and
# SQ_INSTS_VALU/SALU/WAVES (never mixed with trace domains), then tools/profile_summary.py
# writes profiles/<TAG>_{kernel_stats.csv,hbm_traffic.json,summary.md}; bench.py's relit legs
# take their roofline's VALU count and traffic from the newest such record of their workload.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="$1"; CFG="$2"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
for s in kt fetch write valu; do rm -rf "$R/gpurun_out/prof_${TAG}_$s"; done
B="$R/bench.py --config $CFG --fused-only --streams 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_kt" \
  -- python3 $B --steps 10 --warmup 3 > "$R/gpurun_out/prof_${TAG}_kt.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/prof_${TAG}_kt.log"; exit $rc; }
for P in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES:valu"; do
  CT="${P%%:*}"; S="${P##*:}"
  timeout -k 10 400 rocprofv3 --pmc $CT --output-format csv -d "$R/gpurun_out/prof_${TAG}_$S" \
    -- python3 $B --steps 2 --warmup 1 --event-steps 1 > "$R/gpurun_out/prof_${TAG}_$S.log" 2>&1
  rc=$?; echo "$S rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/prof_${TAG}_$S.log"; exit $rc; }
done
python3 "$R/tools/profile_summary.py" "$TAG"
