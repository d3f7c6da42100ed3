#!/bin/bash
# full-size parity, an A/B of the cfg 2 kernel against a staged older tree
# (rl-rust_amd/exp/r01tree, optional), then rocprofv3 evidence (trace stats +
# separate PMC passes) for every SURVEY §8(d) bench workload.  Stops at the
# first failing GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_fullsize.py} -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_full.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -d rl-rust_amd/exp/r01tree ] && [ -n "$AB" ]; then
  for i in 1 2; do
    (cd rl-rust_amd/exp/r01tree && timeout -k 10 120 python -u bench.py --no-cpu-baseline > ../../../gpurun_out/ab_old_$i.log 2>&1) || exit 1
    timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/ab_head_$i.log 2>&1 || exit 1
    python - <<PY
import json
for n in ("old", "head"):
    d = [json.loads(l) for l in open(f"gpurun_out/ab_{n}_$i.log") if l.startswith("{")][-1]
    print(n, "$i", "%.4g" % d["value"], "kern_ms %.4f" % d["roofline"]["kernel_avg_ms"])
PY
  done
fi
for spec in ${PROF:-2:0 2:1 3:0 4:0 5:0}; do
  c=${spec%%:*}; s=${spec##*:}
  ROUND=${RPFX:-r02}_cfg${c}_s$s BENCH_ARGS="--config $c --slippery $s" bash scripts/profile.sh > gpurun_out/profile_cfg${c}_s$s.log 2>&1 || { rc=$?; echo "profile cfg$c s$s rc=$rc"; tail -5 gpurun_out/profile_cfg${c}_s$s.log; exit $rc; }
  echo "profiled cfg$c slippery=$s"
done
