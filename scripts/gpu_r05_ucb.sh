#!/bin/bash
# UCB selection / probabilities: per-action branches (RLAMD_UCB_PRED=0) vs predicated
# (1), on cfg 3 (Taxi UCB + expected SARSA, the NaN regime) and cfg 8 (Taxi UCB +
# Q-learning, finite Q): parity on the bench-size fixtures, then alternating benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS="es0 es1" TESTS=tests/test_gpu_fullsize.py KSEL="cfg3" REPS=3 BENCH_ARGS="--config 3" bash scripts/gpu_abn.sh || exit $?
VARS="ql0 ql1" TESTS=tests/test_gpu_fullsize.py KSEL="cfg8" REPS=3 BENCH_ARGS="--config 8" bash scripts/gpu_abn.sh || exit $?
