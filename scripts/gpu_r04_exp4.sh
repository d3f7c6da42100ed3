#!/bin/bash
# round-4 experiment 4: cfg 4's pair-pool sweep — the last rounds in chunks of 2 / 1
# (c4tail) and no tag rewrite for items that keep their slot (c4t2), against the same
# sources with the old chunking (c4base): parity at bench geometry, then A/B at 2^17
# and 2^19 lanes; and the LDS microbench (gathers + 64-bit atomics) under PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/exp4
for v in c4tail c4t2 c4u2; do
  RLAMD_LIB=$PWD/rl-rust_amd/exp/librlamd_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_longrun.py -m gpu -x -q -k cfg4 --timeout 300 --timeout-method thread > gpurun_out/exp4/pytest_$v.log 2>&1 || { tail -20 gpurun_out/exp4/pytest_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/exp4/pytest_$v.log)"
done
VARS="c4base c4tail c4t2 c4u2" REPS=3 BENCH_ARGS="--config 4" bash scripts/gpu_abn.sh || exit 1
VARS="c4base c4tail c4t2 c4u2" REPS=2 BENCH_ARGS="--config 4 --lanes 524288" bash scripts/gpu_abn.sh || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES \
  -d gpurun_out/exp4/lds -o run --output-format csv -- rl-rust_amd/exp/lds_gather > gpurun_out/exp4/lds.log 2>&1 || { tail -5 gpurun_out/exp4/lds.log; exit 1; }
grep kernel gpurun_out/exp4/lds.log
