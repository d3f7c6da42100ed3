#!/bin/bash
# full bench lines (cpu_baseline included) for the given SURVEY cfgs -> gpurun_out/bench_cfg<c>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CONFIGS:-2 3 4 5}; do
  timeout -k 10 300 python -u bench.py --config $c ${BENCH_ARGS} > gpurun_out/bench_cfg$c.log 2>&1 || { rc=$?; tail -5 gpurun_out/bench_cfg$c.log; exit $rc; }
  grep '^{' gpurun_out/bench_cfg$c.log | tail -1 > gpurun_out/bench_cfg$c.json
  python -c "
import json; d=json.load(open('gpurun_out/bench_cfg$c.json')); r=d['roofline']; cb=d['cpu_baseline']
print('cfg$c', '%.4g'%d['value'], 'kern_ms %.4f'%r['kernel_avg_ms'], r['bound'], d['dtype'], 'cpu %.4g'%cb['value'], 'mc %.4g x%d'%(cb['multi_core']['value'], cb['multi_core']['cores']))"
done
