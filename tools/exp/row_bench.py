"""Row-structure experiments at the C2 shape (see row_kernels.hip). Experiment only."""
import ctypes, os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import vsiquantization_amd  # noqa  (torch first, one HIP runtime)
HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "row_kernels.so"))
scl = ctypes.CDLL(os.path.join(HERE, "stream_kernels.so"))
dev = torch.device("cuda:0")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
R, L = 1024, 9216
N = R * L
SL = 8
xs = [torch.randn(N, device=dev) for _ in range(SL)]
ys = [torch.empty(N, device=dev) for _ in range(SL)]
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


cfgs = [("copy nt u1 g2048", lambda i: scl.exp_copy(P(xs[i % SL].data_ptr()), P(ys[i % SL].data_ptr()), ctypes.c_int64(N // 4), 2048, 1, 1, st))]
for bs in (256, 512, 1024):
    for rpb in (1, 2, 4, 8):
        for red in (0, 1):
            for lds in ((0, 48 * 1024, 64 * 1024) if rpb == 1 else (0,)):
                if lds and bs == 256:
                    continue
                if lib.exp_row(P(xs[0].data_ptr()), P(ys[0].data_ptr()), R, L, bs, rpb, red, lds, st) != 0:
                    continue
                cfgs.append((f"row bs{bs} rpb{rpb} red{red} lds{lds // 1024}k",
                             (lambda bs, rpb, red, lds: lambda i: lib.exp_row(
                                 P(xs[i % SL].data_ptr()), P(ys[i % SL].data_ptr()), R, L, bs, rpb, red, lds, st))(bs, rpb, red, lds)))
torch.cuda.synchronize()
res = {}
for rnd in range(3):
    for name, fn in cfgs:
        res.setdefault(name, []).append(t(fn))
for name, v in res.items():
    us = sorted(v)[1]
    print(f"{name:32s} {us:8.2f} us  {2 * N * 4 / us / 1e3:8.1f} GB/s")
