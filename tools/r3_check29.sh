#!/bin/bash
# round 3: cfg4 iteration on one stream under the kernel trace
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/kt_train"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_train" \
  -- python3 "$R/tools/train_kernels.py" 10 > "$R/gpurun_out/kt_train.log" 2>&1 || { tail -5 "$R/gpurun_out/kt_train.log"; exit 1; }
grep "one stream" "$R/gpurun_out/kt_train.log"
