cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2; do
for kb in 64 70 76; do
  RLAMD_TRC_KB=$kb timeout -k 10 200 python -u bench.py --config 4 --no-cpu-baseline > gpurun_out/trc_$kb.log 2>&1 || { tail -5 gpurun_out/trc_$kb.log; exit 1; }
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/trc_$kb.log') if l.startswith('{')][-1]
print('kb $kb', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], d['config']['groups_per_cu'], d['config']['lds_bytes_per_group'])"
done
done
