#!/bin/bash
# bench lines for every SURVEY §8(d) workload -> gpurun_out/bench_<key>.json
# (cfg 2 with the CPU baseline, as the driver runs it); stops at the first failure
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {   # key, bench args
  timeout -k 10 300 python -u bench.py $2 > gpurun_out/bench_$1.log 2>&1 || { rc=$?; tail -5 gpurun_out/bench_$1.log; exit $rc; }
  grep '^{' gpurun_out/bench_$1.log | tail -1 > gpurun_out/bench_$1.json
  python -c "
import json; d=json.load(open('gpurun_out/bench_$1.json')); r=d['roofline']
print('$1', '%.4g'%d['value'], 'kern_ms %.4f'%r['kernel_avg_ms'], 'frac %.3f'%r['frac'], 'issue', r.get('issue_frac'), 'clamp', d.get('q_clamp_hits'))"
}
run cfg2 ""
run cfg2_slippery "--config 2 --slippery 1 --no-cpu-baseline"
run cfg3 "--config 3 --no-cpu-baseline"
run cfg4 "--config 4 --no-cpu-baseline"
run cfg5 "--config 5 --no-cpu-baseline"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { rc=$?; tail -5 gpurun_out/smoke.log; exit $rc; }
tail -1 gpurun_out/smoke.log
