#!/bin/bash
# cfg 4 at BASELINE's 2^19 lanes on one GPU: the pair-pool LDS share per group
# (RLAMD_TRC_KB) against occupancy; default = the host's choice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for kb in default ${KBS:-8 16 24 32 48 64}; do
  if [ $kb = default ]; then unset RLAMD_TRC_KB; else export RLAMD_TRC_KB=$kb; fi
  timeout -k 10 200 python -u bench.py --config 4 --lanes ${LANES:-524288} --no-cpu-baseline > gpurun_out/trc_$kb.log 2>&1 || { tail -5 gpurun_out/trc_$kb.log; exit 1; }
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/trc_$kb.log') if l.startswith('{')][-1]
print('trc_kb $kb', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], 'groups/CU', d['config']['groups_per_cu'], 'lds', d['config']['lds_bytes_per_group'])"
done
