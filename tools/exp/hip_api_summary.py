"""Summarize a rocprofv3 --hip-trace CSV (hip_api_trace.csv): per HIP API function, calls,
total and mean host time, and calls / time per step (steps = argv[2]).  Used to compare
the public-API C2 step's host work with torch's trivial (x * 1.0).backward(g) step
(tools/exp/api_trace.py under MODE=api / MODE=torch).
usage: python tools/exp/hip_api_summary.py DIR_OR_CSV STEPS"""
import collections
import csv
import glob
import os
import sys


def rows(path):
    files = [path] if path.endswith(".csv") else glob.glob(os.path.join(path, "**", "*hip_api_trace.csv"),
                                                            recursive=True)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                yield r


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    acc = collections.defaultdict(lambda: [0, 0.0])
    for r in rows(path):
        name = r.get("Function") or r.get("Name") or r.get("Kernel_Name")
        t0, t1 = float(r["Start_Timestamp"]), float(r["End_Timestamp"])
        acc[name][0] += 1
        acc[name][1] += (t1 - t0) * 1e-3   # ns -> us
    tot = sum(v[1] for v in acc.values())
    print(f"{'function':40s} {'calls':>8s} {'calls/step':>10s} {'us/call':>8s} {'us/step':>8s}")
    for name, (n, us) in sorted(acc.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{name:40s} {n:8d} {n / steps:10.2f} {us / n:8.2f} {us / steps:8.2f}")
    print(f"{'TOTAL HIP API':40s} {sum(v[0] for v in acc.values()):8d} {'':10s} {'':8s} {tot / steps:8.2f}")


if __name__ == "__main__":
    main()
