"""Store gate: wall-clock (auto / f x read_bytes at 7.5 TB/s) vs arrival-released
(VSIQ_TUNE_GATE_ARRIVE p %) on the C2 per-channel K3 forward and STE backward, plus a
one-round K1 (fused ReLU act fq) shape.  Experiment only; events over back-to-back
launches, median of ROUNDS."""
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


def setmode(m):
    kind, v = m
    if kind == "clk":
        assert lib.vsiq_set_tuning(H.TUNE_GATE_ARRIVE, 0) == 0
        assert lib.vsiq_set_tuning(H.TUNE_STORE_GATE, v) == 0
    else:
        assert lib.vsiq_set_tuning(H.TUNE_STORE_GATE, -1) == 0
        assert lib.vsiq_set_tuning(H.TUNE_GATE_ARRIVE, v) == 0


shapes = [tuple(int(d) for d in s.split("x")) for s in os.environ.get(
    "SHAPES", "1024x1024x3x3 512x1024x3x3 2048x1024x3x3 1024x512x3x3").split()]
ROUNDS = int(os.environ.get("ROUNDS", "5"))
PCTS = [int(v) for v in os.environ.get("PCTS", "60 75 85 90 95 100").split()]
for shp in shapes:
    W = type("W", (bench.C2PerChannel,), {"shape": shp})(dev, 8, 0)
    SL = len(W.slots)
    est = W.n * 4 / 75000  # ticks of 1.0 x read_bytes / 7.5 TB/s
    modes = [("clk", 0), ("clk", -1)] + [("clk", int(f * est)) for f in (0.9, 1.2, 1.4)] + \
        [("arr", p) for p in PCTS]
    out = {}
    for rnd in range(ROUNDS):
        for m in modes:
            setmode(m)
            out.setdefault(("fwd", m), []).append(t(lambda i: W.f_fwd(*W.slots[i % SL]["fwd"])))
            out.setdefault(("bwd", m), []).append(t(lambda i: W.f_bwd(*W.slots[i % SL]["bwd"])))
    for k in ("fwd", "bwd"):
        row = "  ".join(f"{m[0]}{m[1]}:{sorted(out[(k, m)])[len(out[(k, m)]) // 2]:6.2f}" for m in modes)
        print(f"{str(shp):20s} {k} {row}", flush=True)
    del W
    torch.cuda.empty_cache()
setmode(("clk", -1))
