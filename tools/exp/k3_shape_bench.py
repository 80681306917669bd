"""K3 at C2 across workgroup shapes (VSIQ_TUNE_PC_BLOCK x VSIQ_TUNE_PC_ROWS_PER_BLOCK), each
with its store gate tuned online first.  Experiment only."""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa
from vsiquantization_amd import _hip as H
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
lib = H.lib()
W = bench.C2PerChannel(dev, 8, 0)
SL = len(W.slots)
fw = lambda i: W.f_fwd(*W.slots[i % SL]["fwd"])


def t(fn, reps=64):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(8):
        assert fn(i) == 0
    torch.cuda.synchronize(); s.record()
    for i in range(reps):
        fn(i)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for rnd in range(2):
    for bs, rpb in [(256, 1), (256, 2), (512, 1), (1024, 1), (512, 2)]:
        H.set_tuning(H.TUNE_PC_BLOCK, bs)
        H.set_tuning(H.TUNE_PC_ROWS_PER_BLOCK, rpb)
        torch.cuda.synchronize()
        assert lib.vsiq_gate_reset() == 0
        n = 0
        while n < 400:
            for _ in range(16):
                fw(n); n += 1
            torch.cuda.synchronize()
            if H.gate_tuning_pending() == 0:
                break
        rep = [l for l in H.gate_report().splitlines() if l.startswith("k3")]
        best = rep[0].split("best=")[1].split()[0] if rep else "-"
        ts = sorted(t(fw) for _ in range(5))
        H.set_tuning(H.TUNE_STORE_GATE, 0)
        t0 = sorted(t(fw) for _ in range(5))[2]
        H.set_tuning(H.TUNE_STORE_GATE, -1)
        print(f"bs {bs:4d} rpb {rpb}: tuned gate {best:>4s} -> {ts[2]:6.2f} us (min {ts[0]:.2f}); no gate {t0:6.2f} us", flush=True)
