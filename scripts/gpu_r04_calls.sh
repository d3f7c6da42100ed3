#!/bin/bash
# round 4: the per-call Agent surface tests, the whole GPU suite, then a cfg 2 bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_agent_calls.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_agent_calls.log 2>&1
rc=$?; echo "agent calls rc=$rc"; tail -15 gpurun_out/pytest_agent_calls.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_longrun.py::test_bench_window_matches_oracle[cfg2] --deselect "tests/test_gpu_longrun.py::test_bench_window_matches_oracle[cfg2_slippery]" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_cfg2.log 2>&1 || { tail -20 gpurun_out/bench_cfg2.log; exit 1; }
grep '^{' gpurun_out/bench_cfg2.log | tail -1
