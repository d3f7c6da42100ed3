#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
for pad in 0 90000; do
  RLAMD_MIN_SMEM=$pad timeout -k 10 200 python bench.py --no-cpu-baseline --lanes 131072 --steps 64 --warmup 2 > gpurun_out/smem_$pad.log 2>&1 || { tail -5 gpurun_out/smem_$pad.log; exit 1; }
  python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/smem_$pad.log') if l.startswith('{')][-1]
print('pad $pad', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], d['q_check']['match'])"
done
done
for pad in 0 45000; do
  RLAMD_MIN_SMEM=$pad timeout -k 10 200 python bench.py --no-cpu-baseline --lanes 262144 --steps 64 --warmup 2 > gpurun_out/smem2_$pad.log 2>&1 || { tail -5 gpurun_out/smem2_$pad.log; exit 1; }
  python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/smem2_$pad.log') if l.startswith('{')][-1]
print('2^18 pad $pad', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'])"
done
