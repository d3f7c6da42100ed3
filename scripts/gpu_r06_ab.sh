#!/bin/bash
# round 6 A/B: VARS builds (rl-rust_amd/exp), parity on the cfg 2 fixtures first,
# then alternating bench runs at the 2^17-lane shard and at 2^20
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TESTS="${TESTS:-tests/test_gpu_longrun.py tests/test_gpu_global_q.py tests/test_gpu_fullsize.py}"
export KSEL="${KSEL:-cfg2 and not slippery and not f64 and not L2M and not L4M and not L8M}"
REPS=${REPS:-3} BENCH_ARGS="--lanes 131072 --steps 64 --warmup 2" bash scripts/gpu_abn.sh || exit $?
unset TESTS
REPS=${REPS2:-2} BENCH_ARGS="--steps 64 --warmup 2" bash scripts/gpu_abn.sh || exit $?
