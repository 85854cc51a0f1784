#!/bin/bash
# A/B of tile-pass variants (round 3): base, bwd at 5 waves, bwd one body per reach mask (4 / 5
# waves), fwd one body per reach mask; each twice, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=relightable3dgaussians-w_amd/lib
STEPS=30 bash tools/variants.sh base v5=$L/v5/libgsr.so sw4=$L/sw4/libgsr.so sw5=$L/sw5/libgsr.so fsw=$L/fsw/libgsr.so \
  base v5=$L/v5/libgsr.so sw4=$L/sw4/libgsr.so sw5=$L/sw5/libgsr.so fsw=$L/fsw/libgsr.so
