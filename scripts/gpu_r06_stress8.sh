#!/bin/bash
# round 6: the peer-read merge over many launches at 8 ranks sharing the GPU (the
# driver's largest SCALE shape): cfg 2's strong split for 1500 launches, cfg 3
# (f64 + UCB counters) 300, cfg 4 (f64 traces) 300 — every rank's digest compared
# (q_check.ranks_agree); any peer wait past its timeout fails the run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/stress8
for c in "2 1500" "3 300" "4 300"; do
  set -- $c
  RLAMD_COLLECTIVE=peer RLAMD_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --config $1 --gpus 8 --steps $2 --warmup 2 --no-cpu-baseline > gpurun_out/stress8/cfg$1.json 2> gpurun_out/stress8/cfg$1.err || { tail -5 gpurun_out/stress8/cfg$1.err; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/stress8/cfg$1.json') if l.startswith('{')][-1])
print('cfg$1', d['n_gpus'], d['steps'], '%.4g'%d['value'], d['config']['merge_path'], json.dumps(d['q_check']))"
done
