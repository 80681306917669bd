"""K3 store gate (VSIQ_TUNE_STORE_GATE) across per-channel weight shapes: gate = f x
read_bytes / 75000 ticks (10 ns). Experiment only."""
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


shapes = [tuple(int(d) for d in s.split("x")) for s in os.environ.get(
    "SHAPES", "1024x1024x3x3 768x1024x3x3 512x1024x3x3 1280x1024x3x3 2048x1024x3x3 1024x512x3x3 "
    "2048x512x3x3 1024x768x3x3 4096x256x3x3 1024x2048x1x1 256x1024x3x3").split()]
ROUNDS = int(os.environ.get("ROUNDS", "3"))
fs = [float(v) for v in os.environ.get("FS", "0 0.6 0.8 0.9 1.0 1.1").split()]
for shp in shapes:
    W = type("W", (bench.C2PerChannel,), {"shape": shp})(dev, 8, 0)
    SL = len(W.slots)
    out = {}
    for rnd in range(ROUNDS):
        for f in fs:
            # f < 0: the automatic gate (-1)
            assert lib.vsiq_set_tuning(H.TUNE_STORE_GATE, -1 if f < 0 else int(f * W.n * 4 / 75000)) == 0
            out.setdefault(("fwd", f), []).append(t(lambda i: W.f_fwd(*W.slots[i % SL]["fwd"])))
            # STE: f = 0 -> the default (auto store defer)
            assert lib.vsiq_set_tuning(H.TUNE_STORE_GATE, int(f * W.n * 4 / 75000) if f > 0 else -1) == 0
            out.setdefault(("bwd", f), []).append(t(lambda i: W.f_bwd(*W.slots[i % SL]["bwd"])))
    for k in ("fwd", "bwd"):
        row = "  ".join(f"f{f}:{sorted(out[(k, f)])[len(out[(k, f)]) // 2]:6.2f}" for f in fs)
        print(f"{str(shp):22s} {k}  {row}   ({W.n * 8 / 1e6:.1f} MB)", flush=True)
    del W
    torch.cuda.empty_cache()
assert lib.vsiq_set_tuning(H.TUNE_STORE_GATE, -1) == 0
