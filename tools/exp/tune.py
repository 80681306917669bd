"""Sweep the vsiq tuning knobs on the bench workloads (interleaved rounds, one process)."""
import itertools, json, os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa
from vsiquantization_amd import _hip as H

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
import vsiquantization_amd  # noqa

def measure(W, steps=64):
    ns = len(W.slots)
    groups = [(g0, min(ns, steps - g0)) for g0 in range(0, steps, ns)]
    for i in range(ns):
        W.launch(i)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in groups]
    torch.cuda.synchronize()
    for (g0, c), ev in zip(groups, evs):
        W.launch_group(g0, c, ev)
    torch.cuda.synchronize()
    f = sum(e[0].elapsed_time(e[1]) for e in evs) / steps * 1e3
    b = sum(e[1].elapsed_time(e[2]) for e in evs) / steps * 1e3
    return f, b

res = {}
c2 = bench.C2PerChannel(dev, 8, 0)
for rnd in range(3):
    for bs, rpb, nt in itertools.product((256, 512, 1024), (1, 2), (0, 1)):
        H.set_tuning(H.TUNE_PC_BLOCK, bs)
        H.set_tuning(H.TUNE_PC_ROWS_PER_BLOCK, rpb)
        H.set_tuning(H.TUNE_NONTEMPORAL, nt)
        res.setdefault(f"c2 bs{bs} rpb{rpb} nt{nt}", []).append(measure(c2))
H.set_tuning(H.TUNE_PC_BLOCK, 0)
H.set_tuning(H.TUNE_PC_ROWS_PER_BLOCK, 0)
H.set_tuning(H.TUNE_NONTEMPORAL, 1)
del c2
torch.cuda.empty_cache()
c3 = bench.C3Lsq(dev, 2, 0)
for rnd in range(3):
    for nt in (0, 1):
        H.set_tuning(H.TUNE_NONTEMPORAL, nt)
        res.setdefault(f"c3 nt{nt}", []).append(measure(c3, steps=16))
for k, v in res.items():
    f = sorted(x[0] for x in v)[len(v) // 2]
    b = sorted(x[1] for x in v)[len(v) // 2]
    print(f"{k:24s} fwd {f:9.2f} us  bwd {b:9.2f} us")
