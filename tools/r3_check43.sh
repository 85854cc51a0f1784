#!/bin/bash
# round 3: tile-pass occupancy re-check after the late changes (forward 5 waves instead of 6,
# backward 5 instead of 4): cfg2 kernel traces
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p relightable3dgaussians-w_amd/lib/base && cp relightable3dgaussians-w_amd/lib/libgsr.so relightable3dgaussians-w_amd/lib/base/
bash tools/kt_variants.sh '--steps 20 --warmup 5 --no-cpu-baseline --no-refalgo --no-train --no-minibatch' base fw5 bw5 base fw5 bw5
