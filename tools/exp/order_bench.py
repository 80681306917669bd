"""Does the STE backward run slower right after the K3 forward? (C2 bench buffers.)"""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa
import vsiquantization_amd  # noqa

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
W = bench.C2PerChannel(dev, 8, 0)
ns = len(W.slots)


def timed(fn, groups=16):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(groups)]
    for g in range(2):
        fn(g)
    torch.cuda.synchronize()
    for g, (a, b) in enumerate(evs):
        a.record(); fn(g); b.record()
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in evs) / groups / ns * 1e3


def fwd8(g):
    for j in range(ns):
        W.f_fwd(*W.slots[j]["fwd"])


def bwd8(g):
    for j in range(ns):
        W.f_bwd(*W.slots[j]["bwd"])


for i in range(ns):
    W.launch(i)
torch.cuda.synchronize()
res = {}
for rnd in range(3):
    res.setdefault("fwd x8 alone", []).append(timed(fwd8))
    res.setdefault("bwd x8 alone", []).append(timed(bwd8))
    # bwd group right after a fwd group (timed: bwd only)
    evs = []
    for g in range(16):
        fwd8(g)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); bwd8(g); b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    res.setdefault("bwd x8 after fwd x8", []).append(sum(a.elapsed_time(b) for a, b in evs) / 16 / ns * 1e3)
    evs = []
    for g in range(16):
        bwd8(g)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fwd8(g); b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    res.setdefault("fwd x8 after bwd x8", []).append(sum(a.elapsed_time(b) for a, b in evs) / 16 / ns * 1e3)
for k, v in res.items():
    print(f"{k:24s} {sorted(v)[1]:8.2f} us/launch")
