"""Mean PMC counter value per dispatch from rocprofv3 --pmc csv output, grouped by
(kernel name, workgroups).  FETCH_SIZE is reported doubled and both in bytes (the gfx950
corrections of tools/pmc_to_traffic.py: KiB units, FETCH_SIZE half-counts 16-B/lane reads).
usage: python tools/exp/pmc_by_grid.py PMC_DIR COUNTER [name-filter ...]"""
import csv
import glob
import statistics
import sys
from collections import defaultdict


def main():
    d, counter, filt = sys.argv[1], sys.argv[2], sys.argv[3:]
    acc = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            if filt and not any(s in name for s in filt):
                continue
            grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
            wg = int(r.get("Workgroup_Size", r.get("Workgroup_Size_X", 1)) or 1)
            acc[(name.split("(")[0][:90], grid // max(wg, 1))].append(float(r["Counter_Value"]))
    mult = 2048.0 if counter == "FETCH_SIZE" else 1024.0
    for (name, wgs), v in sorted(acc.items()):
        print(f"{counter} {name:90s} wgs={wgs:7d} n={len(v):5d} bytes={statistics.mean(v) * mult:14.0f}")


if __name__ == "__main__":
    main()
