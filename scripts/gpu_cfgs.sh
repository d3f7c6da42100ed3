#!/bin/bash
# dist rehearsal tests, then the other SURVEY §8(d) bench lines (+ optional PMC profiles)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_sel.log; [ $rc -eq 0 ] || exit $rc
fi
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_cfg$c.log 2>&1 || { rc=$?; tail -5 gpurun_out/bench_cfg$c.log; exit $rc; }
  grep '^{' gpurun_out/bench_cfg$c.log | tail -1 > gpurun_out/bench_cfg$c.json
  python -c "
import json; d=json.load(open('gpurun_out/bench_cfg$c.json')); r=d['roofline']
print('cfg$c', '%.4g'%d['value'], 'kern_ms %.4f'%r['kernel_avg_ms'], 'frac %.3f'%r['frac'])"
done
for c in ${PROF_CONFIGS}; do
  ROUND=${RPFX:-r02}_cfg$c BENCH_ARGS="--config $c ${PROF_ARGS}" bash scripts/profile.sh > gpurun_out/profile_cfg$c.log 2>&1 || { rc=$?; echo "profile cfg$c rc=$rc"; exit $rc; }
done
