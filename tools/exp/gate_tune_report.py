"""Store-gate tuner consistency: C2 steps (K3 + STE) until the tuner settles, print its
report (median event-timed launch per candidate), reset, repeat; then the back-to-back
time of each chosen gate vs fixed gates.  Experiment only."""
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


def t(fn, reps=64):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(8):
        assert fn(i) == 0
    torch.cuda.synchronize(); s.record()
    for i in range(reps):
        fn(i)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


chosen = []
for rep in range(int(os.environ.get("REPS", "4"))):
    torch.cuda.synchronize()
    assert lib.vsiq_gate_reset() == 0
    n = bench.settle_gates(W)[0]
    print(f"rep {rep}: settled after {n} steps", flush=True)
    r = H.gate_report()
    print(r, flush=True)
    chosen.append([int(l.split("best=")[1].split()[0]) for l in r.splitlines()])
fw = lambda i: W.f_fwd(*W.slots[i % SL]["fwd"])
bw = lambda i: W.f_bwd(*W.slots[i % SL]["bwd"])
for ticks in sorted({c[0] for c in chosen} | {0, 480, 503, 528, 553, 578}):
    lib.vsiq_set_tuning(H.TUNE_STORE_GATE, ticks)
    print(f"fixed {ticks}: fwd {sorted(t(fw) for _ in range(5))[2]:.2f} us", flush=True)
for ticks in sorted({c[1] for c in chosen} | {0, 494, 519, 545, 571}):
    lib.vsiq_set_tuning(H.TUNE_STORE_GATE, ticks)
    print(f"fixed {ticks}: bwd {sorted(t(bw) for _ in range(5))[2]:.2f} us", flush=True)
lib.vsiq_set_tuning(H.TUNE_STORE_GATE, -1)
