"""Per-kernel statistics of bench.py's TIMED REGIONS only, from a rocprofv3 kernel trace.

`bench.py --markers` launches the empty kernel `vsiq_timed_region_marker` right before
(1 workgroup) and right after (2 workgroups) each timed region (vsiq_trace_marker, outside
the wall-clock window).  This tool keeps the dispatches between a begin marker and the next
end marker -- no warm-up, store-gate settle or tuner candidate launches, no self-check --
and reports, per region and kernel, the dispatch count and the mean / median / min / max
duration, so a profiles/ summary can be set beside the bench line's HIP-event averages.

Usage: python tools/timed_region_stats.py <kernel_trace.csv | dir holding one> [out.csv]
(region 1 is the headline timed region; region 2 the same steps in the other launch mode,
bench.py's alt_launch)."""
import csv
import glob
import os
import statistics
import sys

MARK = "vsiq_timed_region_marker"


def _trace_file(p):
    if os.path.isdir(p):
        c = sorted(glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True))
        if not c:
            raise SystemExit(f"no *kernel_trace.csv under {p}")
        return c[0]
    return p


def _grid(r):
    for k in ("Grid_Size_X", "Grid_Size", "grid_size_x"):
        if k in r and r[k] != "":
            return int(float(r[k]))
    return None


def regions(path):
    rows = list(csv.DictReader(open(_trace_file(path), newline="")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if MARK in name:
            g = _grid(r)
            begin = cur is None if g is None else g <= 64   # 1 x 64 lanes: begin; 2 x 64: end
            if begin:
                cur = []
            elif cur is not None:
                out.append(cur)
                cur = None
            continue
        if cur is not None:
            cur.append((name, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return out


def summarize(region):
    by = {}
    for name, d in region:
        by.setdefault(name, []).append(d)
    res = []
    for name, ds in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        res.append({"name": name, "calls": len(ds), "mean_ns": sum(ds) / len(ds),
                    "median_ns": statistics.median(ds), "min_ns": min(ds), "max_ns": max(ds),
                    "total_ns": sum(ds)})
    return res


def main(argv):
    regs = regions(argv[0])
    out = open(argv[1], "w", newline="") if len(argv) > 1 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Region", "Name", "Calls", "MeanNs", "MedianNs", "MinNs", "MaxNs", "TotalNs"])
    for i, reg in enumerate(regs, 1):
        for s in summarize(reg):
            w.writerow([i, s["name"], s["calls"], f"{s['mean_ns']:.1f}", f"{s['median_ns']:.1f}", s["min_ns"],
                        s["max_ns"], s["total_ns"]])
    if not regs:
        print("no complete marker pair in the trace", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
