"""Kernel statistics of a rocprofv3 rocpd database (the default output format of
`rocprofv3 --kernel-trace --stats` without --output-format csv) as the CSV rocprofv3
writes for --stats: Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs.
Usage: python tools/rocpd_stats.py <results.db> [out.csv]"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [(n, k, s, a, 100.0 * s / tot, lo, hi) for n, k, s, a, lo, hi in rows]


def main(argv):
    out = open(argv[1], "w", newline="") if len(argv) > 1 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for r in stats(argv[0]):
        w.writerow(r)


if __name__ == "__main__":
    main(sys.argv[1:])
