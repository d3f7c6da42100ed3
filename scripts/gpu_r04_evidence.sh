#!/bin/bash
# round 4 evidence, part 1 for the current build: the whole GPU suite, smoke, then
# rocprofv3 trace stats + separate PMC passes for every bench workload
# (collect with scripts/collect_counters.py, then part 2: scripts/gpu_r04_bench.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { rc=$?; tail -5 gpurun_out/smoke.log; exit $rc; }
tail -1 gpurun_out/smoke.log
PROF="${PROF:-cfg2 cfg2_slippery cfg2_f64 cfg3 cfg4 cfg4_2p19 cfg5 cfg6 cfg7}" bash scripts/gpu_r04_profile.sh
