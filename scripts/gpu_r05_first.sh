#!/bin/bash
# round 5, first GPU call: the whole -m gpu suite on this build, then the north
# star's strong-scaling shard (2^17 lanes of cfg 2 per GPU) by group size and
# lanes per wave, beside the 2^20-lane N=1 run of the same preset
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -m5 -B20 "Error\|assert" gpurun_out/pytest_gpu.log | tail -60; exit $rc; }
fi
line() { python3 -c "
import json,sys; d=[json.loads(l) for l in open('gpurun_out/sweep.log') if l.startswith('{')][-1]
print(sys.argv[1], '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], 'ms/step %.4f'%d['ms_per_step'],
      'gpc', d['config']['groups_per_cu'], 'q', (d.get('q_check') or {}).get('match'))" "$1"; }
for rep in 1 2; do
  for L in 131072 1048576; do
    for G in 128 256 512; do
      for LPW in 64 32; do
        RLAMD_LPW=$LPW timeout -k 10 120 python3 bench.py --no-cpu-baseline --lanes $L --group $G --steps 20 --warmup 5 \
          > gpurun_out/sweep.log 2>&1 || { tail -5 gpurun_out/sweep.log; exit 1; }
        line "L$L G$G lpw$LPW"
      done
    done
  done
done
