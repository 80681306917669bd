"""Kernel durations and the idle gaps before each kernel from a rocprofv3 kernel trace csv
(experiment): per kernel name, median duration and median gap to the previous kernel's end."""
import csv, statistics, sys, collections

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows = rows[skip:]
dur, gap = collections.defaultdict(list), collections.defaultdict(list)
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][:60]
    dur[name].append((e - s) / 1e3)
    if prev_end is not None:
        gap[name].append((s - prev_end) / 1e3)
    prev_end = e
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"{len(rows)} kernels over {span:.0f} us")
for k in dur:
    g = gap.get(k, [0.0])
    print(f"{k:62s} n={len(dur[k]):5d} dur med {statistics.median(dur[k]):7.2f} us  gap before med "
          f"{statistics.median(g):7.2f} us  mean {statistics.mean(g):7.2f}")
