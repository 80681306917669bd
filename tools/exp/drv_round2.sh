#!/bin/bash
# bench C2 headline: warmup/steps variants interleaved, 3 repetitions.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
summ() { python3 -c "import json;d=json.load(open('$1'));print('$2',round(d['roofline']['frac'],4),{n:round(v['avg_us'],2) for n,v in d['kernels'].items()},d['config']['self_check'])" | tee -a gpurun_out/drv2.txt; }
for rep in 1 2 3; do
  for SW in "20 5" "20 20" "20 100" "200 20" "20 0"; do
    set -- $SW
    timeout -k 10 120 python3 -u bench.py --steps $1 --warmup $2 --extras none --no-api --no-cpu-baseline > gpurun_out/d.json 2>/dev/null || exit $?
    summ gpurun_out/d.json "s$1w$2"
  done
done
