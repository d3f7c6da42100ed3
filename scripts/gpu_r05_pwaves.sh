#!/bin/bash
# cfg 7 private LDS kernel: lanes per wave x waves per block (RLAMD_PRIV_LPW /
# RLAMD_PRIV_WAVES; LDS caps a CU at ~96 CliffWalking lanes either way): the
# private parity cases first on the variant library, then bench sweeps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/rl-rust_amd/exp/librlamd_pw.so
for w in 1 2; do
  RLAMD_PRIV_WAVES=$w RLAMD_PRIV_LPW=16 RLAMD_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "cw-q" > gpurun_out/pytest_pw_$w.log 2>&1
  rc=$?; echo "waves $w pytest rc=$rc: $(tail -1 gpurun_out/pytest_pw_$w.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/pytest_pw_$w.log | head -5; exit $rc; }
done
one() {   # tag, lpw, waves
  RLAMD_PRIV_LPW=$2 RLAMD_PRIV_WAVES=$3 RLAMD_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --config 7 --steps 16 --warmup 1 --timing-every 1 > gpurun_out/pw_$1.log 2>&1 || { tail -5 gpurun_out/pw_$1.log; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/pw_$1.log') if l.startswith('{')][-1]
print('$1', '%.4g'%d['value'], 'kern_ms %.3f'%d['roofline']['kernel_avg_ms'])"
}
for i in 1 2; do
  one l8w4 8 4
  one l16w2 16 2
  one l32w1 32 1
  one l8w2 8 2
  one l16w1 16 1
  one l4w4 4 4
done
