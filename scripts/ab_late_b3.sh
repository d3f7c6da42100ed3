#!/bin/bash
# GPU parity suite on the in-tree build, then A/B of the late step barrier
# (in-tree) against a Taxi TU built without it (exp/librlamd_tx0.so) on cfg 3,
# and cfg 2 / cfg 5 on the in-tree build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_tests.sh || exit $?
for i in 1 2; do
  for c in "3 base" "3 tx0" "2 base" "5 base"; do
    set -- $c
    if [ $2 = base ]; then L=$PWD/rl-rust_amd/lib/librlamd.so; else L=$PWD/rl-rust_amd/exp/librlamd_$2.so; fi
    RLAMD_LIB=$L timeout -k 10 200 python -u bench.py --config $1 --no-cpu-baseline > gpurun_out/ab_$2.log 2>&1 || { tail -5 gpurun_out/ab_$2.log; exit 1; }
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ab_$2.log') if l.startswith('{')][-1]
print('cfg$1 $2', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'])"
  done
done
