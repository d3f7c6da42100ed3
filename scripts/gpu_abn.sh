#!/bin/bash
# A/B/n of experiment builds rl-rust_amd/exp/librlamd_<v>.so (VARS="a b ..."; "base" =
# the in-tree library): optional parity tests on each (TESTS, -k KSEL), then REPS
# rounds of alternating bench runs (BENCH_ARGS), one line per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
lib_of() { if [ "$1" = base ]; then echo $PWD/rl-rust_amd/lib/librlamd.so; else echo $PWD/rl-rust_amd/exp/librlamd_$1.so; fi; }
if [ -n "$TESTS" ]; then
  for w in $VARS; do
    RLAMD_LIB=$(lib_of $w) timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread ${KSEL:+-k "$KSEL"} > gpurun_out/pytest_ab_$w.log 2>&1
    rc=$?; echo "$w pytest rc=$rc: $(tail -1 gpurun_out/pytest_ab_$w.log)"; [ $rc -eq 0 ] || { grep -m5 -B5 "Error\|assert" gpurun_out/pytest_ab_$w.log | head -40; exit $rc; }
  done
fi
for i in $(seq ${REPS:-3}); do
  for w in $VARS; do
    RLAMD_LIB=$(lib_of $w) timeout -k 10 200 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_$w.log 2>&1 || { tail -5 gpurun_out/ab_$w.log; exit 1; }
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ab_$w.log') if l.startswith('{')][-1]
print('$w', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'])"
  done
done
