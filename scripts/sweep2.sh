#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "--sync 64 --warmup 3" "--sync 64 --warmup 60" "--sync 64 --warmup 200" "--sync 16 --warmup 800" "--sync 256 --warmup 50"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 $cfg > gpurun_out/sweep_tmp.json 2>/dev/null || { echo "fail $cfg"; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep_tmp.json')); print('$cfg', '%.3e'%d['value'], 'kern_ms %.3f'%d['roofline']['kernel_avg_ms'], 'steps/launch %.3g'%d['config']['env_steps_per_launch'])"
done
