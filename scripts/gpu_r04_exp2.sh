#!/bin/bash
# round-4 experiment 2: step-loop segment shares from the stamped diagnostic builds
# (exp/librlamd_st<cfg>.so, -DRLAMD_STAMPS=1), then the distribution test
# (device streams vs the ChaCha12 reference loop).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/exp2
for c in 2 3 4 5; do
  RLAMD_LIB=$PWD/rl-rust_amd/exp/librlamd_st$c.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --config $c --steps 8 > gpurun_out/exp2/st$c.log 2>&1 || { tail -5 gpurun_out/exp2/st$c.log; exit 1; }
  grep rlamd_stamps gpurun_out/exp2/st$c.log | sed "s/^/cfg$c /"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_distribution.py -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/exp2/dist.log 2>&1
rc=$?; grep -E "mean|negative|passed|failed|Error" gpurun_out/exp2/dist.log | head -40; exit $rc
