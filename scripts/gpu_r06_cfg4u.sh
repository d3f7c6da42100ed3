#!/bin/bash
# cfg 4 in the library kernel: sweep width U 4 (base4) against U 8 (u8, -DRLAMD_SWEEP_U=8),
# at 2^17 and 2^19 lanes — does the isolated replay's U 8 gain (scripts/pool_sweep.hip) transfer?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS="base4 u8" TESTS="tests/test_gpu_fullsize.py tests/test_gpu_global_q.py" KSEL="cfg4" REPS=3 \
  BENCH_ARGS="--config 4" bash scripts/gpu_abn.sh || exit $?
echo "--- 2^19 lanes"
VARS="base4 u8" REPS=3 BENCH_ARGS="--config 4 --lanes 524288" bash scripts/gpu_abn.sh || exit $?
