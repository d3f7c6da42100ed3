#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of the default bench,
# then separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ) — never combined
# with runtime or sys tracing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r01}
O=gpurun_out/prof_$R
mkdir -p $O
B="bench.py --no-cpu-baseline --steps 20 --warmup 5 ${BENCH_ARGS}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B > $O/trace.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT"; do
  n=$(echo $c | tr ' ' '_')
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $c -d $O/pmc_$n -o run --output-format csv -- python3 $B > $O/pmc_$n.log 2>&1 || { echo "pmc $c failed rc=$?"; tail -5 $O/pmc_$n.log; }
done
ls -R $O | head -50
