"""Deferred store phase (VSIQ_TUNE_STORE_DEFER) on the product K3 / STE across per-channel
weight shapes. Experiment only."""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa
import vsiquantization_amd  # noqa
from vsiquantization_amd import _hip as H
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
lib = H.lib()


def t(fn, reps=64):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(8):
        assert fn(i) == 0
    torch.cuda.synchronize(); s.record()
    for i in range(reps):
        fn(i)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


shapes = [(1024, 1024, 3, 3), (768, 1024, 3, 3), (512, 1024, 3, 3), (1280, 1024, 3, 3), (2048, 1024, 3, 3),
          (1024, 512, 3, 3), (2048, 512, 3, 3), (1024, 768, 3, 3), (4096, 256, 3, 3), (1024, 2048, 1, 1)]
units = (0, 4, 6, 8, 10, 12, 16)
for shp in shapes:
    W = type("W", (bench.C2PerChannel,), {"shape": shp})(dev, 8, 0)
    SL = len(W.slots)
    out = {}
    for rnd in range(3):
        for u in units:
            assert lib.vsiq_set_tuning(6, u) == 0
            out.setdefault(("fwd", u), []).append(t(lambda i: W.f_fwd(*W.slots[i % SL]["fwd"])))
            out.setdefault(("bwd", u), []).append(t(lambda i: W.f_bwd(*W.slots[i % SL]["bwd"])))
    for k in ("fwd", "bwd"):
        row = "  ".join(f"u{u}:{sorted(out[(k, u)])[1]:6.2f}" for u in units)
        print(f"{str(shp):22s} {k}  {row}   ({W.n * 8 / 1e6:.1f} MB)", flush=True)
    del W
    torch.cuda.empty_cache()
assert lib.vsiq_set_tuning(6, -1) == 0
