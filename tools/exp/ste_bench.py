"""STE-backward shape experiments at the C2 size (see ste_exp.hip). Experiment only."""
import ctypes, os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd  # noqa  (torch first, one HIP runtime)
from vsiquantization_amd import _hip as H
HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "ste_exp.so"))
scl = ctypes.CDLL(os.path.join(HERE, "stream_kernels.so"))
dev = torch.device("cuda:0")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
R, L = 1024, 9216
N = R * L
SL = 8
gs = [torch.randn(N, device=dev) for _ in range(SL)]
ys = [torch.empty(N, device=dev) for _ in range(SL)]
ms = [torch.randint(-2**62, 2**62, (R * 4 * 36,), dtype=torch.int64, device=dev) for _ in range(SL)]
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


cfgs = [("copy nt u1 g1024", lambda i: scl.exp_copy(P(gs[i % SL].data_ptr()), P(ys[i % SL].data_ptr()), ctypes.c_int64(N // 4), 1024, 1, 1, st)),
        ("product ste", lambda i: H.lib().vsiq_ste_bwd_f32(P(gs[i % SL].data_ptr()), P(ms[i % SL].data_ptr()), P(ys[i % SL].data_ptr()), ctypes.c_int64(N), None, ctypes.c_int64(0), ctypes.c_double(0.05), st))]
for mm, name in ((0, "mask"), (4, "halves")):
    for su in ((2, 9) if mm == 0 else (1, 2, 3, 4, 8)):
        for lds in (0,):
            cfgs.append((f"ste {name} su{su} lds{lds // 1024}k", (lambda su, mm, lds: lambda i: lib.exp_ste(
                P(gs[i % SL].data_ptr()), P(ms[i % SL].data_ptr()), P(ys[i % SL].data_ptr()),
                ctypes.c_int64(N), ctypes.c_float(0.05), su, mm, st, lds))(su, mm, lds)))
res = {}
for rnd in range(3):
    for name, fn in cfgs:
        res.setdefault(name, []).append(t(fn))
for name, v in res.items():
    us = sorted(v)[1]
    print(f"{name:28s} {us:8.2f} us  {2 * N * 4 / us / 1e3:8.1f} GB/s")
