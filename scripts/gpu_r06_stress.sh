#!/bin/bash
# round 6: the peer-read merge over many launches — 4 ranks sharing the GPU, 400
# launches of cfg 2's strong split and 100 of cfg 5's (f64 MAX + SUM), every rank's
# digest compared (q_check.ranks_agree)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/stress
for c in "2 400" "5 100"; do
  set -- $c
  RLAMD_COLLECTIVE=peer RLAMD_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --config $1 --gpus 4 --steps $2 --warmup 2 --no-cpu-baseline > gpurun_out/stress/cfg$1.json 2> gpurun_out/stress/cfg$1.err || { tail -5 gpurun_out/stress/cfg$1.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/stress/cfg$1.json').read().splitlines()[-1])
print('cfg$1', d['n_gpus'], d['steps'], '%.4g'%d['value'], d['config']['merge_path'], json.dumps(d['q_check']))"
done
