#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=relightable3dgaussians-w_amd/lib
BENCH_ARGS="--config cfg5 --no-minibatch" STEPS=10 bash tools/variants.sh base g512=$L/g512/libgsr.so g256=$L/g256/libgsr.so base g512=$L/g512/libgsr.so g256=$L/g256/libgsr.so
STEPS=30 bash tools/variants.sh base g512=$L/g512/libgsr.so base g512=$L/g512/libgsr.so
