#!/bin/bash
# quick GPU experiment: the throughput-variant parity tests, then the cfg2 bench
# (and optionally others) — each step under its own time limit, stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "throughput or shared_mode or private_mode" > gpurun_out/exp_pytest.log 2>&1 || { tail -30 gpurun_out/exp_pytest.log; exit 1; }
tail -1 gpurun_out/exp_pytest.log
for c in ${CONFIGS:-2}; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/exp_bench_$c.json 2>&1 || { tail -5 gpurun_out/exp_bench_$c.json; exit 1; }
  python -c "
import json,sys
for l in open('gpurun_out/exp_bench_$c.json'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('cfg$c', '%.4g'%d['value'], 'kern_ms %.4f'%r['kernel_avg_ms'], 'frac %.3f'%r['frac'], 'ms/step %.4f'%d['ms_per_step'])"
done
