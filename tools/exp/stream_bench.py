"""Streaming ceilings at C2 size (37.7 MB in, 37.7 MB out) vs the product kernels.
Run under rocprofv3 --kernel-trace --stats for exact durations."""
import ctypes, os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import vsiquantization_amd  # noqa
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "stream_kernels.so"))
dev = torch.device("cuda:0")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
N = 1024 * 1024 * 9
SL = 8
xs = [torch.randn(N, device=dev) for _ in range(SL)]
ys = [torch.empty(N, device=dev) for _ in range(SL)]
out = torch.zeros(1, device=dev)
P = ctypes.c_void_p
def t(fn, reps=64):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(8): fn(i)
    torch.cuda.synchronize(); s.record()
    for i in range(reps): fn(i)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3
res = {}
for grid in (1024, 2048, 4096, 8192, 9216):
    for nt in (0, 1):
        for un in (1, 4):
            us = t(lambda i: lib.exp_copy(P(xs[i % SL].data_ptr()), P(ys[i % SL].data_ptr()), ctypes.c_int64(N // 4), grid, nt, un, st))
            res[f"copy g{grid} nt{nt} u{un}"] = (us, 2 * N * 4 / us / 1e3)
    us = t(lambda i: lib.exp_read(P(xs[i % SL].data_ptr()), P(out.data_ptr()), ctypes.c_int64(N // 4), grid, st))
    res[f"read g{grid}"] = (us, N * 4 / us / 1e3)
    us = t(lambda i: lib.exp_write(P(ys[i % SL].data_ptr()), ctypes.c_int64(N // 4), grid, st))
    res[f"write g{grid}"] = (us, N * 4 / us / 1e3)
us = t(lambda i: ys[i % SL].copy_(xs[i % SL]))
res["torch copy_"] = (us, 2 * N * 4 / us / 1e3)
big = [torch.randn(N * 16, device=dev) for _ in range(2)]
bo = [torch.empty(N * 16, device=dev) for _ in range(2)]
us = t(lambda i: lib.exp_copy(P(big[i % 2].data_ptr()), P(bo[i % 2].data_ptr()), ctypes.c_int64(N * 4), 8192, 0, 4, st), reps=16)
res["copy 16x size g8192"] = (us, 2 * N * 16 * 4 / us / 1e3)
for k, (us, gbs) in res.items():
    print(f"{k:28s} {us:8.2f} us (events/launch, incl. gaps) {gbs:8.1f} GB/s")
