#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE csv passes into per-launch HBM bytes.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are
in KiB; FETCH_SIZE counts exactly half of the bytes of a wide (16 B/lane) coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B/lane stores.
Usage: pmc_to_traffic.py OUT.json workload=FETCH_DIR,WRITE_DIR [...]
"""
import collections
import csv
import glob
import json
import sys

KERNEL_KEYS = {  # kernel-name fragment -> bench.py kernel label
    "k_pc_observe_fq<": "pc_observe_fq_fwd",
    "k_ste_bwd<": "ste_bwd",
    "k_fq_fwd<": "fq_fwd",
    "k_lsq_bwd<": "lsq_bwd",
}


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            for frag, label in KERNEL_KEYS.items():
                if frag in r["Kernel_Name"]:
                    acc[label].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    out = sys.argv[1]
    res = {"note": "HBM bytes per launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 corrections)"}
    for arg in sys.argv[2:]:
        wl, dirs = arg.split("=")
        fdir, wdir = dirs.split(",")
        fetch, write = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
        res[wl] = {k: {"fetch_bytes": 2 * fetch[k] * 1024, "write_bytes": write.get(k, 0.0) * 1024,
                       "hbm_bytes_per_launch": 2 * fetch[k] * 1024 + write.get(k, 0.0) * 1024}
                   for k in fetch}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
