#!/bin/bash
# round 5 final library: GPU suite + smoke + cfg 6/7 bench lines, then the cfg 7
# private LDS shapes again (lanes per wave x waves per block) on the in-tree library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r05_tests2.sh || exit $?
one() {   # tag, lpw, waves
  RLAMD_PRIV_LPW=$2 RLAMD_PRIV_WAVES=$3 timeout -k 10 300 python3 bench.py --no-cpu-baseline --config 7 --steps 16 --warmup 1 --timing-every 1 > gpurun_out/pwf_$1.log 2>&1 || { tail -5 gpurun_out/pwf_$1.log; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/pwf_$1.log') if l.startswith('{')][-1]
print('$1', '%.4g'%d['value'], 'kern_ms %.3f'%d['roofline']['kernel_avg_ms'])"
}
for i in 1 2; do
  one l8w4 8 4
  one l16w2 16 2
  one l16w1 16 1
  one l8w2 8 2
  one l4w4 4 4
done
