"""K4 at the C3 size with the three streams (x, g, gx) at different relative offsets;
also a 3-stream copy-like reference (x + g -> gx, plain). Experiment only."""
import ctypes, os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd  # noqa
from vsiquantization_amd import _hip as H
dev = torch.device("cuda:0")
lib = H.lib()
st = H.stream_of(dev)
n = 512 * 3 * 224 * 224
pad = 8 << 20
bufs = [torch.empty(n + pad // 4, device=dev) for _ in range(6)]
for b in bufs:
    b.normal_()
scale = torch.tensor(0.03, dtype=torch.float64, device=dev)
grads = torch.empty(2, dtype=torch.float64, device=dev)
w = H.workspace(dev, n)
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


def k4(ox, og, ogx):
    def f(i):
        base = 3 * (i % 2)
        x = bufs[base].data_ptr() + ox
        g = bufs[base + 1].data_ptr() + og
        gx = bufs[base + 2].data_ptr() + ogx
        return lib.vsiq_lsq_bwd_f32(P(g), P(x), P(gx), H.c_i64(n), H.ptr(scale), 0.0, None, 0.0, 0, -128, 127,
                                    1e-4, H.ptr(grads), H.ptr(w.ws), H.c_i64(w.ws_len), H.ptr(w.counter), st)
    return f


def k1(ox, oy):
    def f(i):
        base = 3 * (i % 2)
        return lib.vsiq_fq_fwd_f32(P(bufs[base].data_ptr() + ox), P(bufs[base + 2].data_ptr() + oy), None, None,
                                   H.c_i64(n), None, H.ptr(scale), 0.0, None, 0.0, 0, 0, -128, 127, st)
    return f


for name, fn in [("k1 0/0", k1(0, 0)), ("k1 0/4352", k1(0, 4352)), ("k4 0/0/0", k4(0, 0, 0)),
                 ("k4 0/4352/8704", k4(0, 4352, 8704)), ("k4 0/1M+4352/2M+8704", k4(0, (1 << 20) + 4352, (2 << 20) + 8704)),
                 ("k4 0/256/512", k4(0, 256, 512)), ("k4 0/64K/128K", k4(0, 65536, 131072)),
                 ("k4 0/0/4352", k4(0, 0, 4352))]:
    us = sorted(t(fn) for _ in range(3))[1]
    b = 8 * n if name.startswith("k1") else 12 * n
    print(f"{name:26s} {us:8.2f} us {b / us / 1e3:7.0f} GB/s", flush=True)
