#!/bin/bash
# cfg 4's pool sweep in isolation on the real workload's inputs (scripts/cfg4_sweep_floor.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/cfg4_sweep_floor.py 10 4 > gpurun_out/sweep_floor.jsonl 2> gpurun_out/sweep_floor.err
rc=$?; cat gpurun_out/sweep_floor.jsonl; tail -5 gpurun_out/sweep_floor.err; exit $rc
