#!/bin/bash
# cfg 4 at 2^19 lanes: lanes per wave (RLAMD_LPW 64 = the host's choice there, 32)
# and the pair-pool LDS share (RLAMD_TRC_KB), alternated
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for v in "64 def" "32 def" "32 20" "64 24"; do
    set -- $v
    if [ $2 = def ]; then unset RLAMD_TRC_KB; else export RLAMD_TRC_KB=$2; fi
    RLAMD_LPW=$1 timeout -k 10 200 python -u bench.py --config 4 --lanes 524288 --no-cpu-baseline > gpurun_out/lpw.log 2>&1 || { tail -5 gpurun_out/lpw.log; exit 1; }
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/lpw.log') if l.startswith('{')][-1]
print('lpw $1 trc $2', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], 'groups/CU', d['config']['groups_per_cu'], 'lds', d['config']['lds_bytes_per_group'])"
  done
done
