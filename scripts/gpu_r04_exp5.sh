#!/bin/bash
# round-4 experiment 5: cfg 2's merge inside the train kernel (the last group folds
# and applies; exp c2fuse) against the separate k_fold_apply (c2nofuse), same sources:
# parity at bench geometry (2 and 65 launches), then A/B in both command shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/exp5
RLAMD_LIB=$PWD/rl-rust_amd/exp/librlamd_c2fuse.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_longrun.py -m gpu -x -q -k cfg2 --timeout 300 --timeout-method thread > gpurun_out/exp5/pytest.log 2>&1 || { tail -20 gpurun_out/exp5/pytest.log; exit 1; }
echo "c2fuse parity: $(tail -1 gpurun_out/exp5/pytest.log)"
VARS="c2nofuse c2fuse" REPS=3 BENCH_ARGS="" bash scripts/gpu_abn.sh || exit 1
VARS="c2nofuse c2fuse" REPS=3 BENCH_ARGS="--steps 20 --warmup 5" bash scripts/gpu_abn.sh || exit 1
