#!/bin/bash
# bench sweep over (sync_every, group_size, warmup) for the headline workload
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for args in "${@:-"--sync 64 --warmup 60"}"; do
  out=$(timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 $args 2>&1) || { echo "FAIL $args"; echo "$out" | tail -5; exit 1; }
  echo "$args $(echo "$out" | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.3e kern_ms %.3f" % (d["value"], d["roofline"]["kernel_avg_ms"]))')"
done
