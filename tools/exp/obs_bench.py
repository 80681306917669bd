"""K2 observer variants (VSIQ_TUNE_OBS_KERNEL / _OBS_GRID) at the C5 layer sizes. Experiment only."""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd  # noqa
from vsiquantization_amd import _hip as H
dev = torch.device("cuda:0")
lib = H.lib()
st = H.stream_of(dev)


def t(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(4):
        assert fn(i) == 0
    torch.cuda.synchronize(); s.record()
    for i in range(reps):
        fn(i)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


W = H.workspace(dev, 1 << 28)
ws, cnt = W.ws, W.counter
stats = torch.zeros(16, dtype=torch.float64, device=dev)
rmm = torch.zeros(2, device=dev)
qp = torch.zeros(4, dtype=torch.float64, device=dev)
variants = [("oneshot", 1, 0), ("pf4 g1024", 2, 1024), ("pf4 g2048", 2, 2048), ("pf4 g512", 2, 512),
            ("pf4 g256", 2, 256), ("plain8 g1024", 3, 1024), ("plain8 g2048", 3, 2048),
            ("plain8 g512", 3, 512), ("plain8 g256", 3, 256), ("plain4 g1024", 4, 1024), ("plain4 g512", 4, 512)]
for n in (52428800, 26214400, 13107200, 6553600, 3276800, 1638400):
    sl = max(2, min(8, (1200 << 20) // (4 * n)))
    xs = [torch.randn(n, device=dev) for _ in range(sl)]
    reps = max(16, min(200, (8 << 30) // (4 * n)))
    row = []
    ref = None
    for name, k, g in variants:
        H.set_tuning(H.TUNE_OBS_KERNEL, k); H.set_tuning(H.TUNE_OBS_GRID, g)
        f = lambda i: lib.vsiq_act_observe_f32(H.ptr(xs[i % sl]), H.c_i64(n), 1, H.ptr(stats), H.ptr(rmm),
                                               H.ptr(qp), 1, 127.0, 1e-8, H.ptr(ws), H.c_i64(ws.numel()),
                                               H.ptr(cnt), st)
        us = sorted(t(f, reps) for _ in range(3))[1]
        torch.cuda.synchronize()
        row.append(f"{name}:{us:6.2f}us/{4 * n / us / 1e3:5.0f}")
    H.set_tuning(H.TUNE_OBS_KERNEL, 0); H.set_tuning(H.TUNE_OBS_GRID, 0)
    print(f"n={n:9d}  " + "  ".join(row), flush=True)
    del xs
