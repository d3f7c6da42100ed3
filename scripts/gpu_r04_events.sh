#!/bin/bash
# round 4: what the per-launch HIP events cost in the driver's command shape
# (--steps 20 --warmup 5): events around every launch, every 4th, none; alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for e in 1 4 0; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --timing-every $e > gpurun_out/ev.log 2>&1 || { tail -5 gpurun_out/ev.log; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/ev.log') if l.startswith('{')][-1]
print('events every $e', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], 'ms_per_step %.4f'%d['ms_per_step'], 'n', d['timing']['kernel_launches_timed'])" | tee -a gpurun_out/events_ab.txt
  done
done
