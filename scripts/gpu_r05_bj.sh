#!/bin/bash
# cfg 5 Blackjack step: hit block + dealer loop (RLAMD_BJ_STEP1=0) vs one draw loop (1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS="bjs0 bjs1" TESTS="tests/test_gpu_fullsize.py tests/test_gpu_longrun.py tests/test_gpu_global_q.py" KSEL="cfg5" REPS=3 \
  BENCH_ARGS="--config 5" bash scripts/gpu_abn.sh || exit $?
