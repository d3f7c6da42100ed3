#!/bin/bash
# round 6: the GPU suite + smoke on this build, then bench lines for cfg 2 (default),
# cfg 2 slippery (f64 since round 6), cfg 6 and cfg 7 (private q_check)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
timeout -k 10 850 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { rc=$?; tail -5 gpurun_out/smoke.log; exit $rc; }
tail -1 gpurun_out/smoke.log
for a in "--config 2" "--config 2 --slippery 1" "--config 6 --timing-every 1" "--config 7 --timing-every 1"; do
  t=$(echo $a | tr -d ' -' )
  timeout -k 10 300 python bench.py $a > gpurun_out/r06/bench_$t.json 2> gpurun_out/r06/bench_$t.err || { tail -5 gpurun_out/r06/bench_$t.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r06/bench_$t.json').read().splitlines()[-1])
print('$t', '%.4g'%d['value'], d['config']['q_repr'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], json.dumps(d['q_check'])[:300])"
done
