#!/bin/bash
# GPU suite, then bench + rocprof evidence. Stops at the first failing GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -1 gpurun_out/bench_default.log
bash scripts/profile.sh > gpurun_out/profile.log 2>&1; rc=$?; echo "profile rc=$rc"; exit $rc
