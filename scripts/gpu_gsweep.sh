cd "${GRAFT_REPO_ROOT:-/root/repo}"
VARS="pin nopin2" REPS=3 bash scripts/gpu_abn.sh || exit 1
for g in 256 1024; do
  RLAMD_LIB=$PWD/rl-rust_amd/exp/librlamd_nopin2.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --group $g > gpurun_out/g$g.log 2>&1 || { tail -5 gpurun_out/g$g.log; exit 1; }
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/g$g.log') if l.startswith('{')][-1]
print('G=$g', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], d['config']['groups_per_cu'])"
done
