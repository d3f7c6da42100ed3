#!/bin/bash
# Round evidence at HEAD in one GPU call: bench lines for every SURVEY §8(d)
# workload with their CPU baselines (gpurun_out/bench_<key>.json), cfg 4 at
# BASELINE's whole 2^19 lanes, rocprofv3 trace stats + separate PMC passes per
# workload (gpurun_out/prof_<RPFX>_cfg<c>_s<s>), then smoke().  Every GPU step
# has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${RPFX:-r03}
if [ -n "$WITH_TESTS" ]; then bash scripts/gpu_tests.sh || exit $?; fi
bench() {   # key, bench args
  timeout -k 10 300 python -u bench.py $2 > gpurun_out/bench_$1.log 2>&1 || { rc=$?; tail -5 gpurun_out/bench_$1.log; exit $rc; }
  grep '^{' gpurun_out/bench_$1.log | tail -1 > gpurun_out/bench_$1.json
  python -c "
import json; d=json.load(open('gpurun_out/bench_$1.json')); r=d['roofline']; c=d.get('cpu_baseline') or {}
print('$1', '%.4g'%d['value'], 'kern_ms %.4f'%r['kernel_avg_ms'], 'bound', r['bound'], 'cpu', c.get('value'))"
}
if [ -z "$SKIP_BENCH" ]; then
  bench cfg2 ""
  bench cfg2_slippery "--config 2 --slippery 1"
  bench cfg3 "--config 3"
  bench cfg4 "--config 4"
  bench cfg4_2p19 "--config 4 --lanes 524288 --no-cpu-baseline"
  bench cfg5 "--config 5"
fi
if [ -z "$SKIP_PROF" ]; then
  for spec in ${PROF:-2:0:cfg2 2:1:cfg2_slippery 3:0:cfg3 4:0:cfg4 5:0:cfg5}; do
    c=$(echo $spec | cut -d: -f1); s=$(echo $spec | cut -d: -f2)
    ROUND=${R}_cfg${c}_s$s BENCH_ARGS="--config $c --slippery $s" bash scripts/profile.sh > gpurun_out/profile_cfg${c}_s$s.log 2>&1 || { rc=$?; echo "profile cfg$c s$s rc=$rc"; tail -5 gpurun_out/profile_cfg${c}_s$s.log; exit $rc; }
    echo "profiled cfg$c slippery=$s"
  done
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { rc=$?; tail -5 gpurun_out/smoke.log; exit $rc; }
tail -1 gpurun_out/smoke.log
