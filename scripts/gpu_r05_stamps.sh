#!/bin/bash
# cfg 2 step-loop segments (scripts/stamps.patch, s_memtime at wave-uniform points):
# st0 no stamps, st1 stamps, st2 stamps + one empty stamp right after each (its own
# cost per location, slots 11-21); three alternations of the default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in st0 st1 st2; do
    RLAMD_LIB=$PWD/rl-rust_amd/exp/librlamd_$v.so timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/st_$v.log 2>&1 || { tail -5 gpurun_out/st_$v.log; exit 1; }
    python3 -c "
import json; L=open('gpurun_out/st_$v.log').read().splitlines()
d=[json.loads(l) for l in L if l.startswith('{')][-1]
s=[l for l in L if l.startswith('rlamd_stamps:')]
print('$v', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], s[-1] if s else '')"
  done
done
