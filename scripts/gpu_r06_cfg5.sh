#!/bin/bash
# cfg 5 (Blackjack double-Q): what one 16-byte row read per step costs, the most
# double-table row summaries could save. base5 = the sources as
# built in-tree (one instantiation, scripts/build_fast.sh); plus1 =
# scripts/cfg5_plus_row.patch: every row load reads one more row of table 1 and folds
# it in through an opaque zero (results unchanged: the parity tests run on it).
# (norb = scripts/cfg5_one_row.patch drops table 1's read instead, but its wrong
# results change the trajectories, so it does not isolate the read: 0.3411 vs 0.3367 ms.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS="base5 plus1" TESTS="tests/test_gpu_fullsize.py tests/test_gpu_global_q.py" KSEL="cfg5" REPS=4 \
  BENCH_ARGS="--config 5" bash scripts/gpu_abn.sh || exit $?
