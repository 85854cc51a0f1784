set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
tools/profile_round.sh r2b > gpurun_out/prof_r2b.out 2>&1; rc=$?; tail -5 gpurun_out/prof_r2b.out; [ $rc -eq 0 ] || exit $rc
tools/configs_round.sh r2b
