#!/bin/bash
# private agents with Q in LDS (k_train_private_lds) and prefetched Dyna planning:
# parity on the Dyna cw-q case and the private cliff-walking parity cases, then
# cfg 7 bench: in-tree library (HBM Q, no prefetch) vs plds with RLAMD_PRIV_LPW 0
# (HBM Q + prefetched planning) / 8 / 16 / 32
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/rl-rust_amd/exp/librlamd_plds.so
one() {   # tag, lib, lpw
  RLAMD_PRIV_LPW=$3 RLAMD_LIB=$2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --config 7 > gpurun_out/plds_$1.log 2>&1 || { tail -5 gpurun_out/plds_$1.log; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/plds_$1.log') if l.startswith('{')][-1]
print('$1', '%.4g'%d['value'], 'kern_ms %.3f'%d['roofline']['kernel_avg_ms'])"
}
for i in 1 2; do
  one lds2 $L 2
  one lds4 $L 4
  one lds8 $L 8
done
# NeuralPolicy (cfg 6) with its parameters in LDS
N=$PWD/rl-rust_amd/exp/librlamd_nlds.so
for lpw in 4 8; do
  RLAMD_PRIV_LPW=$lpw RLAMD_LIB=$N timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "neural" > gpurun_out/pytest_nlds_$lpw.log 2>&1
  echo "nlds lpw $lpw pytest: $(tail -1 gpurun_out/pytest_nlds_$lpw.log)"; grep -E "^FAILED" gpurun_out/pytest_nlds_$lpw.log | head -5
done
oneN() {
  RLAMD_PRIV_LPW=$3 RLAMD_LIB=$2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --config 6 --steps 16 > gpurun_out/nlds_$1.log 2>&1 || { tail -5 gpurun_out/nlds_$1.log; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/nlds_$1.log') if l.startswith('{')][-1]
print('neural $1', '%.4g'%d['value'], 'kern_ms %.3f'%d['roofline']['kernel_avg_ms'])"
}
oneN hbm $N 0
oneN lds2 $N 2
oneN lds4 $N 4
oneN lds8 $N 8
oneN lds16 $N 16
