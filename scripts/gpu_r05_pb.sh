#!/bin/bash
# cfg 7: Dyna planning batch size (RLAMD_PLAN_PB: draws and model reads of PB planning
# steps issued together): the Dyna cw-q parity case per variant, then alternating cfg 7 benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export VARS="${VARS:-pb4 pb8 pb16}"
TESTS="tests/test_gpu_parity.py tests/test_gpu_private_bench.py" KSEL="cw-q or 7" REPS=0 bash scripts/gpu_abn.sh || exit $?
REPS=${REPS:-2} BENCH_ARGS="--config 7 --steps 16 --warmup 1 --timing-every 1" bash scripts/gpu_abn.sh || exit $?
