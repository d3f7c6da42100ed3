#!/bin/bash
# round 6: the fused fixed-point peer merge — parity (dist peer tests, world-1 RCCL
# setup tests, bench --gpus 2 q_check) and the per-launch cost against the generic form
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_dist_gpu.py tests/test_gpu_rccl.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_fused.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_fused.log | head -30; exit $rc; }
timeout -k 10 200 python -u scripts/time_merge.py 2:131072 2 > gpurun_out/merge_latency_fused.jsonl 2> gpurun_out/merge_latency_fused.err || { tail -5 gpurun_out/merge_latency_fused.err; exit 1; }
cat gpurun_out/merge_latency_fused.jsonl
