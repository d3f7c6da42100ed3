#!/bin/bash
# round 6 A/B on cfg 4 (VARS builds): parity on the cfg 4 fixtures, then alternating
# bench runs at 2^17 and 2^19 lanes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TESTS="tests/test_gpu_longrun.py tests/test_gpu_fullsize.py" KSEL="cfg4"
REPS=2 BENCH_ARGS="--config 4 --steps 32 --warmup 2" bash scripts/gpu_abn.sh || exit $?
unset TESTS
REPS=2 BENCH_ARGS="--config 4 --lanes 524288 --steps 32 --warmup 2" bash scripts/gpu_abn.sh
