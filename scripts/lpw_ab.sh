cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for i in 1 2; do
  for v in 64 32; do
    RLAMD_LPW=$v timeout -k 10 200 python -u bench.py --config 4 --no-cpu-baseline > gpurun_out/lpw_$v.log 2>&1 || exit 1
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/lpw_$v.log') if l.startswith('{')][-1]
print('lpw $v', '%.4g'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_avg_ms'], d['config']['groups_per_cu'])"
  done
done
RLAMD_LPW=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_longrun.py -m gpu -x -q -k cfg4 --timeout 200 --timeout-method thread 2>&1 | tail -2
