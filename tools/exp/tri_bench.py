"""2-read/1-write streaming ceiling at the C3 size vs K4. Experiment only."""
import ctypes, os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd  # noqa
from vsiquantization_amd import _hip as H
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "phase_exp.so"))
dev = torch.device("cuda:0")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
n = 512 * 3 * 224 * 224
bufs = [torch.randn(n, device=dev) for _ in range(6)]
P = ctypes.c_void_p


def t(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(3):
        assert fn(i) == 0
    torch.cuda.synchronize(); s.record()
    for i in range(reps):
        fn(i)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for u in (1, 2, 4, 8, 16):
    f = lambda i: lib.exp_tri(P(bufs[3 * (i % 2)].data_ptr()), P(bufs[3 * (i % 2) + 1].data_ptr()),
                              P(bufs[3 * (i % 2) + 2].data_ptr()), ctypes.c_int64(n), u, st)
    us = sorted(t(f) for _ in range(3))[1]
    print(f"tri u{u:2d} {us:8.2f} us {12 * n / us / 1e3:7.0f} GB/s", flush=True)
for u in (1, 2, 4, 8):
    f = lambda i: lib.exp_phase(P(bufs[3 * (i % 2)].data_ptr()), P(bufs[3 * (i % 2) + 2].data_ptr()),
                                ctypes.c_int64(n), 2 if u < 4 else (4 if u == 4 else 9), 0, 0, st)
