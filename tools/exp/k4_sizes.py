"""K4 groups-per-lane (VSIQ_TUNE_LSQ_GROUPS) vs tensor size. Experiment only."""
import ctypes, os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd  # noqa
from vsiquantization_amd import _hip as H
dev = torch.device("cuda:0")
lib = H.lib()
st = H.stream_of(dev)
P = ctypes.c_void_p
scale = torch.tensor(0.03, dtype=torch.float64, device=dev)
grads = torch.empty(2, dtype=torch.float64, device=dev)
H.set_tuning(H.TUNE_LSQ_GROUPS, 2)
w = H.workspace(dev, 110 << 20)
H.set_tuning(H.TUNE_LSQ_GROUPS, 0)


def t(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(3):
        assert fn(i) == 0
    torch.cuda.synchronize(); s.record()
    for i in range(reps):
        fn(i)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for n in (295936, 1048576, 3276800, 6553600, 13107200, 26214400, 52428800, 104857600):
    sl = max(2, min(8, (1600 << 20) // (12 * n)))
    bufs = [torch.randn(n, device=dev) for _ in range(3 * sl)]
    reps = max(10, min(200, (8 << 30) // (12 * n)))
    row = []
    for G in (2, 4, 16):
        H.set_tuning(H.TUNE_LSQ_GROUPS, G)
        f = lambda i: lib.vsiq_act_lsq_bwd_f32(P(bufs[3 * (i % sl)].data_ptr()), P(bufs[3 * (i % sl) + 1].data_ptr()),
                                               P(bufs[3 * (i % sl) + 2].data_ptr()), H.c_i64(n), 1, H.ptr(scale), 0.0,
                                               None, 0.0, 0, 0, 15, 1e-4, H.ptr(grads), H.ptr(w.ws), H.c_i64(w.ws_len),
                                               H.ptr(w.counter), st)
        us = sorted(t(f, reps) for _ in range(3))[1]
        row.append(f"G{G}:{us:7.2f}us/{12 * n / us / 1e3:5.0f}")
    H.set_tuning(H.TUNE_LSQ_GROUPS, 0)
    print(f"n={n:10d} " + "  ".join(row), flush=True)
    del bufs
