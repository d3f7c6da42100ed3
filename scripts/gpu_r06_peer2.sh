#!/bin/bash
# round 6: peer-read merge at 2 and 4 ranks (processes sharing the GPU): parity, latency
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "peer" > gpurun_out/pytest_peer.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_peer.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_peer.log | head -30; exit $rc; }
timeout -k 10 300 python -u scripts/time_peer_merge.py > gpurun_out/peer_latency_w2.jsonl 2> gpurun_out/peer_latency.err || { tail -5 gpurun_out/peer_latency.err; exit 1; }
cat gpurun_out/peer_latency_w2.jsonl
PEER_RANKS=4 timeout -k 10 300 python -u scripts/time_peer_merge.py 2:131072 2:262144 5:131072 > gpurun_out/peer_latency_w4.jsonl 2> gpurun_out/peer_latency4.err || { tail -5 gpurun_out/peer_latency4.err; exit 1; }
cat gpurun_out/peer_latency_w4.jsonl
