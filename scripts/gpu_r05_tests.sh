#!/bin/bash
# round 5: the whole GPU suite and smoke on this build, the per-call timing and the
# merge latency budget
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { rc=$?; tail -5 gpurun_out/smoke.log; exit $rc; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u scripts/time_calls.py > gpurun_out/time_calls.json 2> gpurun_out/time_calls.err || { tail -5 gpurun_out/time_calls.err; exit 1; }
cat gpurun_out/time_calls.json
timeout -k 10 300 python -u scripts/time_merge.py > gpurun_out/merge_latency.jsonl 2> gpurun_out/merge_latency.err || { tail -5 gpurun_out/merge_latency.err; exit 1; }
cat gpurun_out/merge_latency.jsonl
