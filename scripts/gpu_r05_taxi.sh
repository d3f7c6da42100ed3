#!/bin/bash
# Taxi transition word read a step ahead from the HBM table (RLAMD_TAXI_PF) against
# taxi_word's arithmetic: cfg 3 and cfg 8 fixtures per variant, then alternating benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS="tx0c3 tx1c3" TESTS="tests/test_gpu_fullsize.py tests/test_gpu_longrun.py" KSEL="cfg3" REPS=0 bash scripts/gpu_abn.sh || exit $?
VARS="tx0c8 tx1c8" TESTS="tests/test_gpu_fullsize.py tests/test_gpu_longrun.py" KSEL="cfg8" REPS=0 bash scripts/gpu_abn.sh || exit $?
VARS="tx0c3 tx1c3" REPS=3 BENCH_ARGS="--config 3" bash scripts/gpu_abn.sh || exit $?
VARS="tx0c8 tx1c8" REPS=3 BENCH_ARGS="--config 8" bash scripts/gpu_abn.sh || exit $?
