#!/bin/bash
# GPU parity suite (+ optional bench lines): one pytest process, per-test timeout
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
for c in ${CONFIGS}; do
  timeout -k 10 200 python -u bench.py --config $c ${BENCH_ARGS} > gpurun_out/bench_cfg$c.log 2>&1 || { rc=$?; tail -5 gpurun_out/bench_cfg$c.log; exit $rc; }
  grep '^{' gpurun_out/bench_cfg$c.log | tail -1 > gpurun_out/bench_cfg$c.json
  python -c "
import json; d=json.load(open('gpurun_out/bench_cfg$c.json')); r=d['roofline']
print('cfg$c', '%.4g'%d['value'], 'kern_ms %.4f'%r['kernel_avg_ms'], 'frac %.3f'%r['frac'], d.get('config',{}).get('groups_per_cu'))"
done
