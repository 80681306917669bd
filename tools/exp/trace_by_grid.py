"""Per-dispatch kernel durations from a rocprofv3 --kernel-trace CSV, grouped by (kernel
name, grid size): count, median and min duration in us.  Reduces a large trace to a few
lines on the GPU box.  usage: python tools/exp/trace_by_grid.py TRACE_DIR [name-filter ...]"""
import csv
import glob
import statistics
import sys
from collections import defaultdict


def main():
    d, filt = sys.argv[1], sys.argv[2:]
    acc = defaultdict(list)
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            if filt and not any(s in name for s in filt):
                continue
            grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
            wg = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            acc[(name.split("(")[0][:90], grid // max(wg, 1))].append(dur)
    for (name, wgs), v in sorted(acc.items(), key=lambda kv: (kv[0][0], kv[0][1])):
        print(f"{name:90s} wgs={wgs:7d} n={len(v):6d} med={statistics.median(v):8.2f} min={min(v):8.2f} "
              f"sum={sum(v):10.1f}")


if __name__ == "__main__":
    main()
