#!/bin/bash
# End-of-round evidence for the final code: rocprofv3 stats + FETCH/WRITE/VALU passes at cfg2
# and cfg5 (tag $1, default r3u), then the GPU suite, smoke, the default line and the other configurations.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
T="${1:-r3u}"
cd "$R"
tools/profile_round.sh $T > gpurun_out/prof_${T}.out 2>&1 || { echo "profile cfg2 failed"; tail -5 gpurun_out/prof_${T}.out; exit 1; }
tail -3 gpurun_out/prof_${T}.out
tools/profile_round.sh ${T}_cfg5 --config cfg5 > gpurun_out/prof_${T}_cfg5.out 2>&1 || { echo "profile cfg5 failed"; tail -5 gpurun_out/prof_${T}_cfg5.out; exit 1; }
tail -3 gpurun_out/prof_${T}_cfg5.out
cd "$R" && tools/gpu_round.sh || exit $?
tools/configs_round.sh $T
