#!/bin/bash
# round 3: the relit composition test's margins, old vs new shade build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/relightable3dgaussians-w_amd/lib
for v in ${VARIANTS:-old new}; do
  lib=$L/$v/libgsr.so; [ $v = new ] && lib=$L/libgsr.so
  echo "== $v"; GSR_LIB_PATH=$lib timeout -k 10 120 python tools/relit_margin.py || exit 1
done
