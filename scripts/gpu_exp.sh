#!/bin/bash
# experiment loop: GPU parity suite (optional), then bench lines given as ';'-separated arg sets in $BENCHES
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_exp.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_exp.log; [ $rc -eq 0 ] || { grep -m5 -B5 "Error\|assert" gpurun_out/pytest_exp.log | head -40; exit $rc; }
fi
i=0
IFS=';' read -ra B <<< "$BENCHES"
for args in "${B[@]}"; do
  i=$((i+1))
  timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > gpurun_out/exp_$i.log 2>&1 || { rc=$?; echo "bench [$args] rc=$rc"; tail -5 gpurun_out/exp_$i.log; exit $rc; }
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/exp_$i.log') if l.startswith('{')][-1]; r=d['roofline']
print('[$args]', '%.4g'%d['value'], 'kern_ms %.4f'%r['kernel_avg_ms'], 'frac %.3f'%r['frac'], 'occ', d['config'].get('groups_per_cu'), d['config'].get('lds_bytes_per_group'))"
done
