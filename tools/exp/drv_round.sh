#!/bin/bash
# The driver's exact bench command, repeated, plus warmup variants and a per-launch rocprof trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
summ() { python3 -c "import json;d=json.load(open('$1'));print('$2',round(d['roofline']['frac'],4),{n:round(v['avg_us'],2) for n,v in d['kernels'].items()},d['config']['self_check'])" | tee -a gpurun_out/drv.txt; }
for i in 1 2 3; do
  timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 5 --extras none --no-api --no-cpu-baseline > gpurun_out/drv_$i.json 2>/dev/null || exit $?
  summ gpurun_out/drv_$i.json "s20w5"
done
for W in 20 100; do
  timeout -k 10 120 python3 -u bench.py --steps 20 --warmup $W --extras none --no-api --no-cpu-baseline > gpurun_out/drvw.json 2>/dev/null || exit $?
  summ gpurun_out/drvw.json "s20w$W"
done
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_drv -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --extras none --no-api --no-cpu-baseline > gpurun_out/drvp.json 2>/dev/null || exit $?
python3 - <<'PY' | tee -a gpurun_out/drv.txt
import csv, glob
rows = []
for f in glob.glob("gpurun_out/prof_drv/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k3 = [r for r in rows if "k_pc_observe_fq<" in r["Kernel_Name"]]
ste = [r for r in rows if "k_ste_bwd" in r["Kernel_Name"]]
d = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print("K3 per launch us:", [round(d(r), 2) for r in k3])
print("STE per launch us:", [round(d(r), 2) for r in ste])
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(k3, k3[1:])]
print("K3->K3 gaps us:", [round(g, 2) for g in gaps])
PY
