#!/bin/bash
# round-4 experiment 1: (a) the LDS bank-conflict floor of random row gathers
# (scripts/lds_gather.hip); (b) cfg 3's SALU: the one-sided barrier's poll loop
# with s_sleep 1 / 4 / 16 between polls (exp builds c3b / c3s4 / c3s16), bench
# A/B and one SQ_INSTS pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/exp1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES \
  -d gpurun_out/exp1/lds -o run --output-format csv -- rl-rust_amd/exp/lds_gather > gpurun_out/exp1/lds.log 2>&1 || { tail -5 gpurun_out/exp1/lds.log; exit 1; }
cat gpurun_out/exp1/lds.log | grep kernel
VARS="c3b c3s4 c3s16" REPS=2 BENCH_ARGS="--config 3" bash scripts/gpu_abn.sh || exit 1
for v in c3b c3s4 c3s16; do
  RLAMD_LIB=$PWD/rl-rust_amd/exp/librlamd_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    -d gpurun_out/exp1/pmc_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --config 3 > gpurun_out/exp1/pmc_$v.log 2>&1 || { tail -5 gpurun_out/exp1/pmc_$v.log; exit 1; }
  echo "pmc $v done"
done
