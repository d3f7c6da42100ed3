#!/bin/bash
# Taxi + UCB reset drawn one reset ahead (RLAMD_TAXI_RPF) against
# the reset-time draw: cfg 3 and cfg 8 fixtures per variant, then alternating benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS="tr0c3 tr1c3" TESTS="tests/test_gpu_fullsize.py tests/test_gpu_longrun.py tests/test_gpu_parity.py" KSEL="cfg3 or (shared_mode and taxi and expected_sarsa and not traces)" REPS=0 bash scripts/gpu_abn.sh || exit $?
VARS="tr0c8 tr1c8" TESTS="tests/test_gpu_fullsize.py tests/test_gpu_longrun.py tests/test_gpu_parity.py" KSEL="cfg8 or (shared_mode and taxi and qlearning and not traces and not double)" REPS=0 bash scripts/gpu_abn.sh || exit $?
VARS="tr0c3 tr1c3" REPS=3 BENCH_ARGS="--config 3" bash scripts/gpu_abn.sh || exit $?
VARS="tr0c8 tr1c8" REPS=3 BENCH_ARGS="--config 8" bash scripts/gpu_abn.sh || exit $?
