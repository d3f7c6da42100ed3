#!/bin/bash
# round-4 experiment 6: the fused reset's selection reading its row only for
# exploiting lanes (RLAMD_LAZY_ROWS; exp c5lazy / c4lazy against c5base / c4base):
# parity at bench geometry, then A/B on cfg 5 and cfg 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/exp6
for v in "c5lazy cfg5" "c4lazy cfg4"; do
  set -- $v
  RLAMD_LIB=$PWD/rl-rust_amd/exp/librlamd_$1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_longrun.py -m gpu -x -q -k $2 --timeout 300 --timeout-method thread > gpurun_out/exp6/pytest_$1.log 2>&1 || { tail -20 gpurun_out/exp6/pytest_$1.log; exit 1; }
  echo "$1 parity: $(tail -1 gpurun_out/exp6/pytest_$1.log)"
done
VARS="c5base c5lazy" REPS=3 BENCH_ARGS="--config 5" bash scripts/gpu_abn.sh || exit 1
VARS="c4base c4lazy" REPS=3 BENCH_ARGS="--config 4" bash scripts/gpu_abn.sh || exit 1
