#!/bin/bash
# bench lines of this build (counters attach when profiles/counters.json holds this
# build id) + the merge latency budget at world 1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SKIP_TESTS=1 bash scripts/gpu_r04_full.sh || exit $?
timeout -k 10 300 python -u scripts/time_merge.py > gpurun_out/merge_latency.jsonl 2> gpurun_out/merge_latency.err || { tail -5 gpurun_out/merge_latency.err; exit 1; }
cat gpurun_out/merge_latency.jsonl
