#!/bin/bash
# NeuralPolicy parameters in registers (k_train_private_net, RLAMD_NET_REGS): the bin
# shape's parity test on each variant, then alternating cfg 6 bench runs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export VARS="${VARS:-nr0 nr1}"
TESTS="tests/test_gpu_parity.py" KSEL="neural_policy and 0.5" REPS=0 bash scripts/gpu_abn.sh || exit $?
REPS=${REPS:-2} BENCH_ARGS="--config 6 --steps 8 --warmup 1 --timing-every 1" bash scripts/gpu_abn.sh || exit $?
