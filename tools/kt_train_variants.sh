#!/bin/bash
# one-stream cfg4 kernel traces per library variant: tools/kt_train_variants.sh v... (lib/<v>/libgsr.so)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  rm -rf "$R/gpurun_out/ktt_$v"
  GSR_LIB_PATH=$R/relightable3dgaussians-w_amd/lib/$v/libgsr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d "$R/gpurun_out/ktt_$v" -- python3 "$R/tools/train_kernels.py" 10 > "$R/gpurun_out/ktt_$v.log" 2>&1 \
    || { tail -5 "$R/gpurun_out/ktt_$v.log"; exit 1; }
  echo -n "$v: "; grep "one stream" "$R/gpurun_out/ktt_$v.log"
done
