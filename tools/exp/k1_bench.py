"""K1 fused-ReLU forward per launch at C3/C4 sizes (groups-per-lane variants via VSIQ_LIBRARY).
Experiment only."""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd  # noqa
from vsiquantization_amd import _hip as H
dev = torch.device("cuda:0")
lib = H.lib()
st = H.stream_of(dev)
scale = torch.tensor(0.03, dtype=torch.float64, device=dev)
tag = os.environ.get("VSIQ_LIBRARY", "default")[-10:]


def t(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(3):
        assert fn(i) == 0
    torch.cuda.synchronize(); s.record()
    for i in range(reps):
        fn(i)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for n in (26214400, 52428800, 77070336, 104857600):
    sl = max(2, min(8, (1600 << 20) // (8 * n)))
    xs = [torch.randn(n, device=dev) for _ in range(sl)]
    ys = [torch.empty(n, device=dev) for _ in range(sl)]
    f = lambda i: lib.vsiq_act_fq_fwd_f32(H.ptr(xs[i % sl]), H.ptr(ys[i % sl]), None, None, H.c_i64(n), 1, None,
                                          H.ptr(scale), 0.0, None, 0.0, 0, 0, -8, 7, st)
    us = sorted(t(f, 40) for _ in range(3))[1]
    print(f"{tag:12s} n={n:10d} K1 {us:7.2f} us ({8 * n / us / 1e3:5.0f} GB/s)", flush=True)
    del xs, ys
