# Kernel durations inside the public-API C2 loop (ours vs torch's trivial step), from a
# kernel trace of tools/exp/api_timings.py.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_api -o run --output-format csv -- python3 -u tools/exp/api_timings.py > gpurun_out/prof_api.log 2>&1 || { echo "rc=$?"; tail gpurun_out/prof_api.log; exit 1; }
grep ratio gpurun_out/prof_api.log
python3 - <<'PY'
import csv, statistics, collections
rows = list(csv.DictReader(open("gpurun_out/prof_api/run_kernel_trace.csv")))
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"][:90]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:12]:
    print(f"{len(v):6d} calls  median {statistics.median(v):8.2f} us  p10 {sorted(v)[len(v)//10]:8.2f}  {k}")
PY
