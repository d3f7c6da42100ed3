#!/bin/bash
# rocprofv3 evidence for the round-6 bench workloads of this build: kernel-trace
# stats, then separate PMC passes (scripts/profile.sh) into gpurun_out/prof_r06_<key>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in ${PROF:-cfg2 cfg2_slippery cfg2_f64 cfg2_L131072 cfg3 cfg4 cfg4_2p19 cfg5 cfg6 cfg7 cfg8}; do
  case $spec in
    cfg2) a="--config 2" ;;
    cfg2_slippery) a="--config 2 --slippery 1" ;;
    cfg2_f64) a="--config 2 --q-mode f64" ;;
    cfg2_L131072) a="--config 2 --lanes 131072" ;;
    cfg3) a="--config 3" ;;
    cfg4) a="--config 4" ;;
    cfg4_2p19) a="--config 4 --lanes 524288" ;;
    cfg5) a="--config 5" ;;
    cfg6) a="--config 6 --steps 16" ;;
    cfg7) a="--config 7 --steps 16" ;;
    cfg8) a="--config 8" ;;
  esac
  ROUND=r06_$spec BENCH_ARGS="$a" bash scripts/profile.sh > gpurun_out/profile_$spec.log 2>&1 || { rc=$?; echo "profile $spec rc=$rc"; tail -5 gpurun_out/profile_$spec.log; exit $rc; }
  echo "profiled $spec $(date +%T)"
done
