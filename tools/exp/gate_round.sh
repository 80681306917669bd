#!/bin/bash
# C2 store-gate sweep + the driver's exact bench command, repeated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
SHAPES="1024x1024x3x3" ROUNDS=3 FS="${FS:-0 0.9 1.0 1.05 1.1 1.15 1.2 1.3 1.45}" timeout -k 10 200 python3 -u tools/exp/gate_bench.py > gpurun_out/gate_sweep.txt 2>&1 || exit $?
for i in 1 2 3 4; do
  timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 5 --extras none --no-api --no-cpu-baseline > gpurun_out/drv_$i.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/drv_$i.json'));print('drv',$i,round(d['roofline']['frac'],4),{n:round(v['avg_us'],2) for n,v in d['kernels'].items()})" | tee -a gpurun_out/gate_sweep.txt
done
