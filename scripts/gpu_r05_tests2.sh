#!/bin/bash
# round 5, second library: the whole GPU suite and smoke, then the cfg 6 / cfg 7 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { rc=$?; tail -5 gpurun_out/smoke.log; exit $rc; }
tail -1 gpurun_out/smoke.log
for c in 6 7; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/bench_cfg$c.log 2>&1 || { tail -5 gpurun_out/bench_cfg$c.log; exit 1; }
  grep '^{' gpurun_out/bench_cfg$c.log | tail -1 > gpurun_out/bench_cfg$c.json
  python -c "
import json; d=json.load(open('gpurun_out/bench_cfg$c.json')); r=d['roofline']
print('cfg$c', '%.4g'%d['value'], 'kern_ms %.4f'%r['kernel_avg_ms'], 'ms/step %.4f'%d['ms_per_step'], r['bound'])"
done
