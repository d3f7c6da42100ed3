#!/bin/bash
# GPU suite, then cfg 4 at the bench's 2^17 lanes and at BASELINE's whole 2^19
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_tests.sh || exit $?
for a in "" "--lanes 524288"; do
  timeout -k 10 200 python -u bench.py --config 4 --no-cpu-baseline $a > gpurun_out/b4.log 2>&1 || { tail -5 gpurun_out/b4.log; exit 1; }
  grep -h "^{" gpurun_out/b4.log | python -c "
import sys, json
d = json.loads(sys.stdin.read()); print('%.4g' % d['value'], d['roofline']['kernel_avg_ms'], d['config']['lanes_per_gpu'])"
done
