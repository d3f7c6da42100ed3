#!/bin/bash
# round 5 bench lines of this build (counters attach when profiles/counters.json holds
# this build id) -> gpurun_out/bench_<key>.json; PROF: profile these first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$PROF" ]; then PROF="$PROF" bash scripts/gpu_r05_profile.sh || exit $?; fi
run() {   # key, bench args
  timeout -k 10 400 python -u bench.py $2 > gpurun_out/bench_$1.log 2>&1 || { rc=$?; tail -5 gpurun_out/bench_$1.log; exit $rc; }
  grep '^{' gpurun_out/bench_$1.log | tail -1 > gpurun_out/bench_$1.json
  python -c "
import json; d=json.load(open('gpurun_out/bench_$1.json')); r=d['roofline']
print('$1', '%.4g'%d['value'], 'kern_ms %.4f'%r['kernel_avg_ms'], 'ms/step %.4f'%d['ms_per_step'], r['bound'], 'frac %.3f'%r['frac'],
      'q', (d.get('q_check') or {}).get('match'), 'cpu', d.get('cpu_baseline',{}).get('value'))"
}
for k in ${BENCH:-cfg2 cfg2_driver cfg2_slippery cfg2_f64 cfg2_L131072 cfg3 cfg4 cfg4_2p19 cfg5 cfg6 cfg7 cfg8}; do
  case $k in
    cfg2) run cfg2 "" ;;
    cfg2_driver) run cfg2_driver "--steps 20 --warmup 5 --no-cpu-baseline" ;;
    cfg2_slippery) run cfg2_slippery "--config 2 --slippery 1" ;;
    cfg2_f64) run cfg2_f64 "--config 2 --q-mode f64" ;;
    cfg2_L131072) run cfg2_L131072 "--config 2 --lanes 131072 --no-cpu-baseline" ;;
    cfg3) run cfg3 "--config 3" ;;
    cfg4) run cfg4 "--config 4" ;;
    cfg4_2p19) run cfg4_2p19 "--config 4 --lanes 524288 --no-cpu-baseline" ;;
    cfg5) run cfg5 "--config 5" ;;
    cfg6) run cfg6 "--config 6" ;;
    cfg7) run cfg7 "--config 7" ;;
    cfg8) run cfg8 "--config 8" ;;
  esac
done
