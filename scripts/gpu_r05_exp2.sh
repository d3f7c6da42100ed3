#!/bin/bash
# round 5 experiments 2: cfg 4 LREC / sweep-width variants; Dyna-Q (cfg 7) lane-major
# private tables vs the in-tree entry-major library, with its HBM traffic (PMC)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VARS="lrec nolrec lrecu2 lrecu8" bash scripts/gpu_r05_cfg4ab.sh || exit $?
VARS="base dyna" TESTS=tests/test_gpu_parity.py KSEL="cw-q" REPS=2 BENCH_ARGS="--config 7" bash scripts/gpu_abn.sh || exit $?
for v in base dyna; do
  lib=$PWD/rl-rust_amd/lib/librlamd.so; [ $v = base ] || lib=$PWD/rl-rust_amd/exp/librlamd_$v.so
  for c in FETCH_SIZE WRITE_SIZE; do
    RLAMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/dyna_$v/$c -o run --output-format csv \
      -- python3 bench.py --no-cpu-baseline --config 7 --steps 8 --warmup 1 > gpurun_out/dyna_${v}_$c.log 2>&1 || { tail -5 gpurun_out/dyna_${v}_$c.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob
for v in ("base", "dyna"):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"gpurun_out/dyna_{v}/{c}/**/*counter_collection.csv", recursive=True)
        rows = [r for r in csv.DictReader(open(f[0])) if "k_train_private" in r["Kernel_Name"]] if f else []
        vals = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == c]
        print(v, c, "launch-records", len(vals), "mean per record", sum(vals) / max(len(vals), 1))
PY
