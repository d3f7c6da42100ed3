#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of the default bench,
# then separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ) — never combined
# with runtime or sys tracing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r01}
O=gpurun_out/prof_$R
mkdir -p $O
B="bench.py --no-cpu-baseline ${BENCH_ARGS}"   # the bench defaults: the same command the driver times
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B > $O/trace.log 2>&1 || exit $?
PASSES=${PASSES:-"FETCH_SIZE WRITE_SIZE SQ_WAVES_SQ_INSTS_VALU_SQ_INSTS_LDS_SQ_INSTS_SALU SQ_WAVE_CYCLES_SQ_WAIT_ANY_SQ_WAIT_INST_ANY_SQ_ACTIVE_INST_ANY_SQ_WAIT_INST_LDS_SQ_ACTIVE_INST_VALU_SQ_ACTIVE_INST_LDS_SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE_SQ_LDS_BANK_CONFLICT_SQ_LDS_IDX_ACTIVE_SQ_INSTS_VMEM_RD_SQ_INSTS_VMEM_WR SQ_INSTS_VALU_ADD_F64_SQ_INSTS_VALU_MUL_F64_SQ_INSTS_VALU_FMA_F64_SQ_INSTS_VALU_TRANS_F64_SQ_INSTS_VALU_INT64_SQ_INSTS_VALU_CVT"}
for n in $PASSES; do
  c=$(echo $n | sed 's/_SQ_/ SQ_/g; s/_GRBM_/ GRBM_/g')
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $c -d $O/pmc_$n -o run --output-format csv -- python3 $B > $O/pmc_$n.log 2>&1 || { rc=$?; echo "pmc $c failed rc=$rc"; tail -5 $O/pmc_$n.log; exit $rc; }
done
ls -R $O | head -50
