#!/bin/bash
# cfg 3 bench line (with its CPU baseline) and rocprofv3 evidence at HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config 3 > gpurun_out/bench_cfg3.log 2>&1 || { tail -5 gpurun_out/bench_cfg3.log; exit 1; }
grep '^{' gpurun_out/bench_cfg3.log | tail -1 > gpurun_out/bench_cfg3.json
python -c "
import json; d=json.load(open('gpurun_out/bench_cfg3.json')); print('cfg3', '%.4g'%d['value'], d['roofline']['kernel_avg_ms'], d['cpu_baseline']['value'])"
ROUND=r03_cfg3_s0 BENCH_ARGS="--config 3" bash scripts/profile.sh > gpurun_out/profile_cfg3_s0.log 2>&1 && echo profiled
