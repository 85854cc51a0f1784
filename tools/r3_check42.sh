#!/bin/bash
# round 3: timing experiment -- cfg4 with the composite forward's host wait for the frame totals
# skipped (lib/nowait; unsafe, timing only) against the in-tree library, same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/relightable3dgaussians-w_amd/lib
for v in base nowait base nowait; do
  echo -n "$v: "; GSR_LIB_PATH=$L/$v/libgsr.so timeout -k 10 200 python tools/train_host.py 30 2>&1 | grep "iterations:" || exit 1
done
