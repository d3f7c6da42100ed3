#!/bin/bash
# PMC passes (one counter set per run) over the pool-sweep replay (scripts/pool_sweep.hip)
# at 2^17 and 2^19 lanes: LDS-array busy cycles, bank conflicts, wave-cycle split
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=${TMPDIR:-/tmp}
mkdir -p gpurun_out/sweep_pmc
IN=$TMPDIR/cfg4_steps.u16
SWEEP_INPUT=$IN timeout -k 10 300 python -u scripts/cfg4_sweep_floor.py 10 4 > gpurun_out/sweep_pmc/capture.log 2>&1 || { tail -5 gpurun_out/sweep_pmc/capture.log; exit 1; }
for tile in 1 4; do
  n=0
  for c in "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"; do
    n=$((n+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/sweep_pmc/t${tile}_p$n -o run --output-format csv -- rl-rust_amd/exp/pool_sweep $IN 131072 64 4 $tile > gpurun_out/sweep_pmc/t${tile}_p$n.log 2>&1 || { rc=$?; echo "pmc tile $tile pass $n rc=$rc"; tail -5 gpurun_out/sweep_pmc/t${tile}_p$n.log; rm -f $IN; exit $rc; }
    echo "tile $tile pass $n ok"
  done
done
rm -f $IN
