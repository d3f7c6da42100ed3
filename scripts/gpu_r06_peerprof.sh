#!/bin/bash
# round 6: kernel-trace stats of the peer-read merge path at world 1 (RLAMD_FORCE_COMM +
# RLAMD_PEER_WORLD1: bench.py's RCCL bootstrap, set_comm's peer setup, every merge
# through k_peer_fold_put / k_peer_reduce_apply) on the north star's 2^17-lane shard
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/peerprof
RLAMD_FORCE_COMM=1 RLAMD_PEER_WORLD1=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/peerprof/trace -o run --output-format csv -- python3 bench.py --lanes 131072 --no-cpu-baseline > gpurun_out/peerprof/trace.log 2>&1 || { tail -5 gpurun_out/peerprof/trace.log; exit 1; }
grep '^{' gpurun_out/peerprof/trace.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['config']['merge_path'], d['config']['collective'])"
find gpurun_out/peerprof -name 'run_kernel_stats.csv' -exec cat {} \;
