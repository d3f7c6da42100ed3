#!/bin/bash
# the driver's round-end sequence on the committed tree: GPU suite, smoke(), bench.py defaults
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rehearsal
timeout -k 10 850 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rehearsal/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/rehearsal/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/rehearsal/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rehearsal/smoke.log 2>&1 || { rc=$?; tail -5 gpurun_out/rehearsal/smoke.log; exit $rc; }
tail -1 gpurun_out/rehearsal/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/rehearsal/bench.log 2>&1 || { rc=$?; tail -5 gpurun_out/rehearsal/bench.log; exit $rc; }
tail -1 gpurun_out/rehearsal/bench.log
