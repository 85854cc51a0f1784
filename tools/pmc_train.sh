#!/bin/bash
# PMC passes (counters only, no trace domains) for the composite tile passes of the cfg4
# training iteration (tools/train_kernels.py on one stream), the same three passes of <= 8 SQ
# counters as tools/pmc_round.sh.  Summarise with
#   python3 tools/pmc_summary.py "gpurun_out/TAG_*/*/*_counter_collection.csv"
#   tools/pmc_train.sh TAG [KERNEL_REGEX] [ITERS]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="${1:-pmc_train}"
KRE="${2:-k_render_(fwd|bwd)_mc}"
ITERS="${3:-2}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
i=0
for CT in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
          "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
          "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf "$R/gpurun_out/${TAG}_$i"
  timeout -k 10 300 rocprofv3 --pmc $CT --kernel-include-regex "$KRE" --output-format csv \
    -d "$R/gpurun_out/${TAG}_$i" -- python3 "$R/tools/train_kernels.py" "$ITERS" > "$R/gpurun_out/${TAG}_$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/${TAG}_$i.log"; exit $rc; }
done
