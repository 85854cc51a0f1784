#!/bin/bash
# round 3: relit features timing (tools/bench_relit.py) per library variant, twice each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/relightable3dgaussians-w_amd/lib
for rep in 1 2; do
for v in ${VARIANTS:-old new}; do
  lib=$L/$v/libgsr.so; [ $v = new ] && lib=$L/libgsr.so
  echo -n "$v: "; GSR_LIB_PATH=$lib timeout -k 10 120 python tools/bench_relit.py 2>&1 | grep "^P=" || exit 1
done
done
