#!/bin/bash
# one process over the same global lane sets and launch counts as gpu_r06_stress8.sh:
# the merged Q's digest must equal the 8-rank peer runs' (exact merges: any rank count)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/stress8
for c in "2 1500 1048576" "3 300 1048576" "4 300 524288"; do
  set -- $c
  timeout -k 10 500 python bench.py --config $1 --lanes $3 --steps $2 --warmup 2 --no-cpu-baseline > gpurun_out/stress8/ref_cfg$1.json 2> gpurun_out/stress8/ref_cfg$1.err || { tail -5 gpurun_out/stress8/ref_cfg$1.err; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/stress8/ref_cfg$1.json') if l.startswith('{')][-1])
print('ref cfg$1', d['n_gpus'], d['steps'], '%.4g'%d['value'], json.dumps(d['q_check']))"
done
