#!/bin/bash
# round 4: the whole GPU suite, smoke, then every bench line (cfg 2 with the CPU
# baseline as the driver runs it; the others with their own) -> gpurun_out/bench_<key>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { rc=$?; tail -5 gpurun_out/smoke.log; exit $rc; }
  tail -1 gpurun_out/smoke.log
fi
run() {   # key, bench args
  timeout -k 10 400 python -u bench.py $2 > gpurun_out/bench_$1.log 2>&1 || { rc=$?; tail -5 gpurun_out/bench_$1.log; exit $rc; }
  grep '^{' gpurun_out/bench_$1.log | tail -1 > gpurun_out/bench_$1.json
  python -c "
import json; d=json.load(open('gpurun_out/bench_$1.json')); r=d['roofline']
print('$1', '%.4g'%d['value'], 'kern_ms %.4f'%r['kernel_avg_ms'], r['bound'], 'frac %.3f'%r['frac'], 'cpu', d.get('cpu_baseline',{}).get('value'))"
}
for k in ${BENCH:-cfg2 cfg2_slippery cfg2_f64 cfg3 cfg4 cfg4_2p19 cfg5 cfg6 cfg7}; do
  case $k in
    cfg2) run cfg2 "" ;;
    cfg2_slippery) run cfg2_slippery "--config 2 --slippery 1 $CPU" ;;
    cfg2_f64) run cfg2_f64 "--config 2 --q-mode f64 $CPU" ;;
    cfg3) run cfg3 "--config 3 $CPU" ;;
    cfg4) run cfg4 "--config 4 $CPU" ;;
    cfg4_2p19) run cfg4_2p19 "--config 4 --lanes 524288 --no-cpu-baseline" ;;
    cfg5) run cfg5 "--config 5 $CPU" ;;
    cfg6) run cfg6 "--config 6 $CPU" ;;
    cfg7) run cfg7 "--config 7 $CPU" ;;
  esac
done
