#!/bin/bash
# bench lines for the given SURVEY cfgs (no CPU baseline): value, kernel ms, occupancy, Q representation
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CONFIGS:-2 3 4 5}; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_cfg$c.log 2>&1 || { rc=$?; tail -5 gpurun_out/bench_cfg$c.log; exit $rc; }
  grep '^{' gpurun_out/bench_cfg$c.log | tail -1 > gpurun_out/bench_cfg$c.json
  python -c "
import json; d=json.load(open('gpurun_out/bench_cfg$c.json')); r=d['roofline']; c=d['config']
print('cfg$c', '%.4g'%d['value'], 'kern_ms %.4f'%r['kernel_avg_ms'], 'ms/step %.4f'%d['ms_per_step'], 'groups/CU', c['groups_per_cu'], 'lds', c['lds_bytes_per_group'], c['q_repr'])"
done
