#!/bin/bash
# cfg 2 run-to-run spread on one box: the default bench 5 times, the driver shape 3 times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/var_$i.log 2>&1 || { tail -3 gpurun_out/var_$i.log; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/var_$i.log') if l.startswith('{')][-1]
print('default', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], 'ms/step %.4f'%d['ms_per_step'])"
done
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/vard_$i.log 2>&1 || { tail -3 gpurun_out/vard_$i.log; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/vard_$i.log') if l.startswith('{')][-1]
print('driver', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], 'ms/step %.4f'%d['ms_per_step'])"
done
