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
import os
import sys

# workload -> [(kernel-name fragment, bench.py kernel label, launches of it per step)];
# a label's bytes per step = sum over its fragments of (mean per dispatch x launches)
KERNEL_KEYS = {
    # C1: K10 (one launch, grid barrier) = one "observe_fq" step; C1_K9=1 runs K9 (K2p
    # records + the fake-quant launch folding them); C1_K2K1=1 K2 + K1 ("observe", "fq_fwd")
    "c1": [("k_observe_fq_grid<", "observe_fq", 1), ("k_observe_part<", "observe_fq", 1), ("k_fold_fq_fwd<", "observe_fq", 1),
           ("k_observe_loop<", "observe", 1), ("k_fq_fwd<", "fq_fwd", 1)],
    # C2: the mask-only K3 instance (MASK true, CODES false); the run also launches the
    # codes variant (9 B/elem, bench's pc_observe_fq_fwd_with_codes), which must not be
    # averaged in (round 2's 1.07x "write excess" was exactly that mix)
    "c2": [(("k_pc_observe_fq<", ", true, false, 256, 1>"), "pc_observe_fq_fwd", 1), ("k_ste_bwd<", "ste_bwd", 1)],
    "c3": [("k_fq_fwd<", "fq_fwd", 1), ("k_lsq_bwd<", "lsq_bwd", 1)],
    # C4: per step 27 fused-ReLU activation launches each way + ONE multi-tensor launch
    # each way for the 27 weights
    "c4": [("k_fq_fwd<", "fwd_all_layers", 27), ("k_lsq_fwd_multi<", "fwd_all_layers", 1),
           ("k_lsq_bwd<", "bwd_all_layers", 27), ("k_lsq_bwd_multi<", "bwd_all_layers", 1)],
    # C5: per calibration batch 27 fused-ReLU K2o launches (calibrate_qat_model's default:
    # y = relu(c) written + the deferred observer's records); round 2/3: one K2m launch
    "c5": [("k_observe_part_out1<", "act_observe_out_all_layers", 27),
           ("k_observe_part_multi<", "observe_all_layers", 1)],
}


def per_kernel(d, counter, keys):
    """Bytes per step of each label: mean counter value per dispatch x launches per step,
    summed over the label's kernels."""
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            for frag, _, _ in keys:
                parts = frag if isinstance(frag, tuple) else (frag,)
                if all(p in r["Kernel_Name"] for p in parts):
                    acc[frag].append(float(r["Counter_Value"]))
    out = collections.defaultdict(float)
    for frag, label, mult in keys:
        if acc[frag]:
            out[label] += sum(acc[frag]) / len(acc[frag]) * mult
    return dict(out)


def main():
    out = sys.argv[1]
    res = {"note": "HBM bytes per launch (C4/C5: per step, all of the label's launches) = "
                   "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 corrections)"}
    if os.path.exists(out):   # keep workloads not re-measured in this call
        old = json.load(open(out))
        res.update({k: v for k, v in old.items() if k != "note"})
    for arg in sys.argv[2:]:
        wl, dirs = arg.split("=")
        fdir, wdir = dirs.split(",")
        keys = KERNEL_KEYS[wl]
        fetch, write = per_kernel(fdir, "FETCH_SIZE", keys), per_kernel(wdir, "WRITE_SIZE", keys)
        res[wl] = {k: {"fetch_bytes": 2 * fetch[k] * 1024, "write_bytes": write.get(k, 0.0) * 1024,
                       "hbm_bytes_per_launch": 2 * fetch[k] * 1024 + write.get(k, 0.0) * 1024}
                   for k in fetch}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
