#!/bin/bash
# A/B of an experimental librlamd build (rl-rust_amd/exp/librlamd_$VAR.so) against
# the in-tree one: parity tests on the variant, then alternating bench runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=rl-rust_amd/exp/librlamd_${VAR:-1}.so
if [ -n "$TESTS" ]; then
  RLAMD_LIB=$PWD/$V timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
  rc=$?; echo "variant pytest rc=$rc"; tail -2 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || { grep -m5 -B5 "Error\|assert" gpurun_out/pytest_ab.log | head -40; exit $rc; }
fi
for i in $(seq ${REPS:-3}); do
  for w in base ${VARS:-${VAR:-1}}; do
    if [ $w = base ]; then L=$PWD/rl-rust_amd/lib/librlamd.so; else L=$PWD/rl-rust_amd/exp/librlamd_$w.so; fi
    RLAMD_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_$w.log 2>&1 || { tail -5 gpurun_out/ab_$w.log; exit 1; }
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ab_$w.log') if l.startswith('{')][-1]
print('$w', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'])"
  done
done
