#!/bin/bash
# round 6: the peer-read merge — world-2 parity (two processes sharing the GPU),
# bench --gpus 2 over it with q_check, then its latency beside RCCL's world-1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_peer.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_peer.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_peer.log | head -30; exit $rc; }
timeout -k 10 300 python -u scripts/time_peer_merge.py > gpurun_out/peer_latency.jsonl 2> gpurun_out/peer_latency.err || { tail -5 gpurun_out/peer_latency.err; exit 1; }
cat gpurun_out/peer_latency.jsonl
timeout -k 10 300 python -u scripts/time_merge.py 2:131072 2 > gpurun_out/merge_latency.jsonl 2> gpurun_out/merge_latency.err || { tail -5 gpurun_out/merge_latency.err; exit 1; }
cat gpurun_out/merge_latency.jsonl
