#!/bin/bash
# One round's evidence: rocprofv3 stats + PMC passes of the bench (profile_round.sh), then the
# secondary configurations (configs_round.sh).  tools/evidence_round.sh <tag>
set -o pipefail
TAG=${1:-r2e}
cd ${GRAFT_REPO_ROOT:-/root/repo}
tools/profile_round.sh $TAG > gpurun_out/prof_$TAG.out 2>&1; rc=$?; tail -5 gpurun_out/prof_$TAG.out; [ $rc -eq 0 ] || exit $rc
tools/configs_round.sh $TAG
