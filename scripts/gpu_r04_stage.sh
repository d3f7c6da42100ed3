#!/bin/bash
# round 4, one GPU call per stage: [TESTS=1: the GPU suite + smoke], then for every
# workload in WL: rocprofv3 evidence (trace stats + separate PMC passes), the
# counters filed for this build (collect_counters.py, on the box), and the bench line
# that attaches them; [MERGE=1: merge latency + the driver's command shape].
# The filed evidence comes back under gpurun_out/sync/ (copy into profiles/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sync
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { rc=$?; tail -5 gpurun_out/smoke.log; exit $rc; }
  tail -1 gpurun_out/smoke.log
fi
for w in $WL; do
  case $w in
    cfg2) c="--config 2" ;;
    cfg2_slippery) c="--config 2 --slippery 1" ;;
    cfg2_f64) c="--config 2 --q-mode f64" ;;
    cfg3) c="--config 3" ;;
    cfg4) c="--config 4" ;;
    cfg4_2p19) c="--config 4 --lanes 524288" ;;
    cfg5) c="--config 5" ;;
    cfg6) c="--config 6" ;;
    cfg7) c="--config 7" ;;
  esac
  PROF=$w bash scripts/gpu_r04_profile.sh || exit 1
  python3 scripts/collect_counters.py gpurun_out/prof_r04_$w r04 $c > gpurun_out/collect_$w.log 2>&1 || { tail -5 gpurun_out/collect_$w.log; exit 1; }
  SKIP_TESTS=1 BENCH=$w bash scripts/gpu_r04_full.sh || exit 1
  cp profiles/r04_*_summary.json profiles/r04_*_kernel_stats.csv profiles/counters.json gpurun_out/sync/ 2>/dev/null
  cp gpurun_out/bench_$w.json gpurun_out/sync/ 2>/dev/null
done
if [ -n "$MERGE" ]; then
  timeout -k 10 300 python -u scripts/time_merge.py > gpurun_out/sync/merge_latency.jsonl 2> gpurun_out/merge_latency.err || { tail -5 gpurun_out/merge_latency.err; exit 1; }
  cat gpurun_out/sync/merge_latency.jsonl
  for i in 1 2 3; do
    for a in "--steps 20 --warmup 5" "--steps 64 --warmup 1"; do
      timeout -k 10 200 python3 bench.py --no-cpu-baseline $a > gpurun_out/shape.log 2>&1 || { tail -5 gpurun_out/shape.log; exit 1; }
      python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/shape.log') if l.startswith('{')][-1]
print('shape $a', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], 'ms_per_step %.4f'%d['ms_per_step'])" | tee -a gpurun_out/sync/shape.txt
    done
  done
fi
