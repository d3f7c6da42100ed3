#!/bin/bash
# bench lines of this build (counters attach when profiles/counters.json holds this
# build id) + the merge latency budget at world 1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SKIP_TESTS=1 bash scripts/gpu_r04_full.sh || exit $?
timeout -k 10 300 python -u scripts/time_merge.py > gpurun_out/merge_latency.jsonl 2> gpurun_out/merge_latency.err || { tail -5 gpurun_out/merge_latency.err; exit 1; }
cat gpurun_out/merge_latency.jsonl
# the driver's own command shape (--steps 20 --warmup 5) beside the default, alternated
for i in 1 2 3; do
  for a in "--steps 20 --warmup 5" "--steps 64 --warmup 1"; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline $a > gpurun_out/shape.log 2>&1 || { tail -5 gpurun_out/shape.log; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/shape.log') if l.startswith('{')][-1]
print('shape $a', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], 'ms_per_step %.4f'%d['ms_per_step'])"
  done
done
