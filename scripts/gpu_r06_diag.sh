#!/bin/bash
# round 6 diagnostics (wrong results by construction, timing only): the cfg 2 kernel
# without its late barrier (diagA) / without its contributions barrier (diagB)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPS=3 BENCH_ARGS="--lanes 131072 --steps 64 --warmup 2" VARS="base0 diagA diagB" bash scripts/gpu_abn.sh || exit $?
REPS=2 BENCH_ARGS="--steps 64 --warmup 2" VARS="base0 diagA diagB" bash scripts/gpu_abn.sh
