#!/bin/bash
# A/B per bench config: for each CFG=base:run pair run the cfg's parity tests on both, then
# alternate bench runs (--config N).  PAIRS="3:c3base:c3run 4:c4base:c4run"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pr in $PAIRS; do
  c=${pr%%:*}; rest=${pr#*:}; a=${rest%%:*}; b=${rest#*:}
  for w in $a $b; do
    RLAMD_LIB=$PWD/rl-rust_amd/exp/librlamd_$w.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_longrun.py -m gpu -x -q --timeout 300 --timeout-method thread -k "cfg$c" > gpurun_out/pytest_ab_$w.log 2>&1
    rc=$?; echo "$w pytest rc=$rc: $(tail -1 gpurun_out/pytest_ab_$w.log)"; [ $rc -eq 0 ] || { grep -m3 -B3 "Error\|assert" gpurun_out/pytest_ab_$w.log | head -20; exit $rc; }
  done
  for i in $(seq ${REPS:-3}); do
    for w in $a $b; do
      RLAMD_LIB=$PWD/rl-rust_amd/exp/librlamd_$w.so timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/ab_$w.log 2>&1 || { tail -5 gpurun_out/ab_$w.log; exit 1; }
      python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ab_$w.log') if l.startswith('{')][-1]
print('cfg$c $w', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'])"
    done
  done
done
