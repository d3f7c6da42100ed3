#!/bin/bash
# round 6 final library: one bench line per workload (counters from profiles/counters.json
# attach: same library), the driver's command shape, and --gpus 2 over the peer merge
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06b
run() {  # tag, args...
  local t=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/r06b/bench_$t.json 2> gpurun_out/r06b/bench_$t.err || { tail -5 gpurun_out/r06b/bench_$t.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r06b/bench_$t.json').read().splitlines()[-1])
r=d['roofline']; q=d.get('q_check') or {}
print('$t', '%.4g'%d['value'], d['config'].get('q_repr'), 'kern %.4f'%r['kernel_avg_ms'], r.get('bound'), 'frac %.3f'%r['frac'], 'fx', q.get('fixture'), q.get('match'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
}
run cfg2 --config 2
run cfg2_driver --config 2 --steps 20 --warmup 5
run cfg2_slippery --config 2 --slippery 1
run cfg2_f64 --config 2 --q-mode f64
run cfg2_L131072 --config 2 --lanes 131072 --no-cpu-baseline
run cfg3 --config 3
run cfg4 --config 4
run cfg4_2p19 --config 4 --lanes 524288 --no-cpu-baseline
run cfg5 --config 5
run cfg6 --config 6 --timing-every 1
run cfg7 --config 7 --timing-every 1
run cfg8 --config 8
RLAMD_COLLECTIVE=peer RLAMD_DIST_BACKEND=gloo run cfg2_gpus2_peer --gpus 2 --steps 20 --warmup 5
