#!/bin/bash
# cfg 4 pair-pool sweep variants (RLAMD_POOL_BF / REC16 / LREC): parity on the
# cfg 4 fixtures (2 launches at bench size, the 65-launch bench window at 2^17
# and 2^19 lanes), then alternating bench runs at both lane counts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export VARS="${VARS:-base bf bfrec bflrec all3}"
TESTS="tests/test_gpu_fullsize.py tests/test_gpu_longrun.py" KSEL="cfg4" REPS=0 bash scripts/gpu_abn.sh || exit $?
REPS=${REPS:-3} BENCH_ARGS="--config 4" bash scripts/gpu_abn.sh || exit $?
REPS=${REPS:-3} BENCH_ARGS="--config 4 --lanes 524288" bash scripts/gpu_abn.sh || exit $?
