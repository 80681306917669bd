"""Load/store phase experiments at the C2 size (see phase_exp.hip). Experiment only."""
import ctypes, os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa
import vsiquantization_amd  # noqa
HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "phase_exp.so"))
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
W = bench.C2PerChannel(dev, 8, 0)
SL = len(W.slots)
N = W.n
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = ctypes.c_void_p


def t(fn, reps=64):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(8):
        assert fn(i) == 0
    torch.cuda.synchronize(); s.record()
    for i in range(reps):
        fn(i)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


cfgs = [("K3 product", lambda i: W.f_fwd(*W.slots[i % SL]["fwd"])),
        ("STE product", lambda i: W.f_bwd(*W.slots[i % SL]["bwd"]))]
for bar, sl in ((1, 0), (1, 64), (1, 80), (1, 96)):
    cfgs.append((f"ste su9 bar{bar} sleep{sl}", (lambda bar, sl: lambda i: lib.exp_ste_phase(
        P(W.slots[i % SL]["g"].data_ptr()), P(W.slots[i % SL]["mask"].data_ptr()),
        P(W.slots[i % SL]["gx"].data_ptr()), ctypes.c_int64(1024), ctypes.c_int64(W.rowlen),
        P(W.slots[i % SL]["scale"].data_ptr()), bar, sl, st))(bar, sl)))
print("wallclock kHz", lib.exp_wallclock_khz(), flush=True)
for gate, ticks in [(2, 0)] + [(1, t) for t in (300, 400, 500, 550, 600, 650, 700, 800)]:
    cfgs.append((f"ste gate{gate} ticks{ticks}", (lambda gate, ticks: lambda i: lib.exp_ste_gate(
        P(W.slots[i % SL]["g"].data_ptr()), P(W.slots[i % SL]["mask"].data_ptr()),
        P(W.slots[i % SL]["gx"].data_ptr()), ctypes.c_int64(1024), ctypes.c_int64(W.rowlen),
        P(W.slots[i % SL]["scale"].data_ptr()), gate, ctypes.c_uint32(ticks), st))(gate, ticks)))
for su in (9,):
    for mode in (2,):
        for sl in (80,):
            cfgs.append((f"phase su{su} mode{mode} sleep{sl}", (lambda su, mode, sl: lambda i: lib.exp_phase(
                P(W.slots[i % SL]["x"].data_ptr()), P(W.slots[i % SL]["y"].data_ptr()), ctypes.c_int64(N),
                su, mode, sl, st))(su, mode, sl)))
res = {}
for rnd in range(5):
    for name, fn in cfgs:
        res.setdefault(name, []).append(t(fn))
for name, v in res.items():
    us = sorted(v)[2]
    print(f"{name:28s} {us:8.2f} us  {2 * N * 4 / us / 1e3:8.1f} GB/s", flush=True)
