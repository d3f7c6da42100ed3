#!/bin/bash
# round-4 experiment 3: cfg 3 with Taxi's start sums in LDS (exp/librlamd_c3cdf.so):
# cfg 3 parity at bench geometry, A/B against the in-tree library, stamped shares.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/exp3
RLAMD_LIB=$PWD/rl-rust_amd/exp/librlamd_c3cdf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_longrun.py -m gpu -x -q -k cfg3 --timeout 300 --timeout-method thread > gpurun_out/exp3/pytest.log 2>&1 || { tail -20 gpurun_out/exp3/pytest.log; exit 1; }
tail -1 gpurun_out/exp3/pytest.log
VARS="base c3cdf" REPS=3 BENCH_ARGS="--config 3" bash scripts/gpu_abn.sh || exit 1
RLAMD_LIB=$PWD/rl-rust_amd/exp/librlamd_st3c.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --config 3 --steps 8 > gpurun_out/exp3/st3c.log 2>&1 || { tail -5 gpurun_out/exp3/st3c.log; exit 1; }
grep rlamd_stamps gpurun_out/exp3/st3c.log
