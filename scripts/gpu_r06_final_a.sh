#!/bin/bash
# round 6 final library, part A: the whole GPU suite + smoke, per-call timing,
# merge latency (local / RCCL world 1 / peer-read at 2 and 4 ranks)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
timeout -k 10 850 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/final/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/final/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { rc=$?; tail -5 gpurun_out/final/smoke.log; exit $rc; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 120 python -u scripts/time_calls.py > gpurun_out/final/time_calls.json 2> gpurun_out/final/time_calls.err || { tail -5 gpurun_out/final/time_calls.err; exit 1; }
timeout -k 10 120 python -u scripts/time_merge.py > gpurun_out/final/merge_latency.jsonl 2> gpurun_out/final/merge_latency.err || { tail -5 gpurun_out/final/merge_latency.err; exit 1; }
timeout -k 10 120 python -u scripts/time_peer_merge.py > gpurun_out/final/peer_latency_w2.jsonl 2> gpurun_out/final/peer_w2.err || { tail -5 gpurun_out/final/peer_w2.err; exit 1; }
PEER_RANKS=4 timeout -k 10 120 python -u scripts/time_peer_merge.py 2:131072 2:262144 5:131072 > gpurun_out/final/peer_latency_w4.jsonl 2> gpurun_out/final/peer_w4.err || { tail -5 gpurun_out/final/peer_w4.err; exit 1; }
cat gpurun_out/final/merge_latency.jsonl gpurun_out/final/peer_latency_w2.jsonl gpurun_out/final/peer_latency_w4.jsonl
