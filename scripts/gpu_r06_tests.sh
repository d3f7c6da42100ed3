#!/bin/bash
# round 6: the whole GPU suite + smoke on this build, then the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { rc=$?; tail -5 gpurun_out/smoke.log; exit $rc; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { rc=$?; tail -5 gpurun_out/bench_default.log; exit $rc; }
tail -1 gpurun_out/bench_default.log
