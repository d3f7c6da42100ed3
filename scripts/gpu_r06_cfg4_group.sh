#!/bin/bash
# cfg 4: learner-group size sweep on the shipped library (bench.py --group), 2^17 and 2^19 lanes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg4g
for L in 131072 524288; do
  for i in 1 2; do
    for g in 128 256 512 1024; do
      timeout -k 10 200 python -u bench.py --config 4 --lanes $L --group $g --no-cpu-baseline > gpurun_out/cfg4g/g$g.log 2>&1 || { tail -5 gpurun_out/cfg4g/g$g.log; exit 1; }
      python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/cfg4g/g$g.log') if l.startswith('{')][-1]
print('L $L G $g', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], 'groups_per_cu', d['config'].get('groups_per_cu'))"
    done
  done
done
