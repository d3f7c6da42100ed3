#!/bin/bash
# bench lines for a list of "cfg|extra args" variants (no CPU baseline): value and kernel time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
while IFS= read -r v; do
  [ -z "$v" ] && continue
  c=${v%%|*}; x=${v#*|}
  i=$((i+1))
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline $x > gpurun_out/var_$i.log 2>&1 || { rc=$?; echo "variant $v failed rc=$rc"; tail -5 gpurun_out/var_$i.log; exit $rc; }
  python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/var_$i.log') if l.startswith('{')][-1]; r=d['roofline']; c=d['config']
print('cfg$c [$x]', '%.4g'%d['value'], 'kern_ms %.4f'%r['kernel_avg_ms'], 'groups/CU', c['groups_per_cu'], 'lds', c['lds_bytes_per_group'])"
done <<< "${VARIANTS}"
