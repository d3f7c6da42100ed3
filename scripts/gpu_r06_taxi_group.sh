#!/bin/bash
# cfg 3 / cfg 8 (Taxi, UCB): learner-group size sweep on the shipped library (bench.py --group)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/taxig
for c in 3 8; do
  for i in 1 2; do
    for g in 256 512 1024; do
      timeout -k 10 200 python -u bench.py --config $c --group $g --no-cpu-baseline > gpurun_out/taxig/g$g.log 2>&1 || { tail -5 gpurun_out/taxig/g$g.log; exit 1; }
      python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/taxig/g$g.log') if l.startswith('{')][-1]
print('cfg $c G $g', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], 'groups_per_cu', d['config'].get('groups_per_cu'))"
    done
  done
done
