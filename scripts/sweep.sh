#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "--group 64 --sync 64" "--group 128 --sync 64" "--group 256 --sync 64" "--group 512 --sync 64" "--group 1024 --sync 64" "--group 64 --sync 256" "--group 256 --sync 256" "--group 64 --sync 16"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 3 $cfg > gpurun_out/sweep_tmp.json 2>/dev/null || { echo "fail $cfg"; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep_tmp.json')); print('$cfg', '%.3e'%d['value'], 'kern_ms %.3f'%d['roofline']['kernel_avg_ms'])"
done
