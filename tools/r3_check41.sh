#!/bin/bash
# round 3: kernel trace of cfg4 on two streams (the bench's schedule) for the GPU's idle time
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/kt_train2"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/kt_train2" \
  -- python3 "$R/tools/train_host.py" 20 > "$R/gpurun_out/kt_train2.log" 2>&1 || { tail -5 "$R/gpurun_out/kt_train2.log"; exit 1; }
grep "iterations:" "$R/gpurun_out/kt_train2.log"
