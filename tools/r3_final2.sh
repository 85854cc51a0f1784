#!/bin/bash
# End-of-round evidence for the final code: rocprofv3 stats + FETCH/WRITE/VALU passes at cfg2
# and cfg5 (tag r3u), then the GPU suite, smoke, the default line and the other configurations.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
tools/profile_round.sh r3u > gpurun_out/prof_r3u.out 2>&1 || { echo "profile cfg2 failed"; tail -5 gpurun_out/prof_r3u.out; exit 1; }
tail -3 gpurun_out/prof_r3u.out
tools/profile_round.sh r3u_cfg5 --config cfg5 > gpurun_out/prof_r3u_cfg5.out 2>&1 || { echo "profile cfg5 failed"; tail -5 gpurun_out/prof_r3u_cfg5.out; exit 1; }
tail -3 gpurun_out/prof_r3u_cfg5.out
cd "$R" && tools/gpu_round.sh || exit $?
tools/configs_round.sh r3u
