"""K4 / K2 per-launch time at C4/C5 layer sizes (fold variants via VSIQ_LIBRARY). Experiment only."""
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
stats = torch.zeros(16, dtype=torch.float64, device=dev)
w = H.workspace(dev, 110 << 20)


def t(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(3):
        assert fn(i) == 0
    torch.cuda.synchronize(); s.record()
    for i in range(reps):
        fn(i)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


tag = os.environ.get("VSIQ_LIBRARY", "default") + os.environ.get("TUNE", "")
for kv in os.environ.get("TUNE", "").split():
    k, v = kv.split("=")
    H.set_tuning(int(k), int(v))
for n in [int(v) for v in os.environ.get('SIZES', '1638400 3276800 6553600 13107200 26214400').split()]:
    sl = max(2, min(8, (1600 << 20) // (12 * n)))
    bufs = [torch.randn(n, device=dev) for _ in range(3 * sl)]
    reps = max(10, min(200, (8 << 30) // (12 * n)))
    f = lambda i: lib.vsiq_act_lsq_bwd_f32(P(bufs[3 * (i % sl)].data_ptr()), P(bufs[3 * (i % sl) + 1].data_ptr()),
                                           P(bufs[3 * (i % sl) + 2].data_ptr()), H.c_i64(n), 1, H.ptr(scale), 0.0,
                                           None, 0.0, 0, 0, 15, 1e-4, H.ptr(grads), H.ptr(w.ws), H.c_i64(w.ws_len),
                                           H.ptr(w.counter), st)
    k4 = sorted(t(f, reps) for _ in range(3))[1]
    g = lambda i: lib.vsiq_act_observe_f32(P(bufs[i % (3 * sl)].data_ptr()), H.c_i64(n), 1, H.ptr(stats), None, None,
                                           1, 127.0, 1e-8, H.ptr(w.ws), H.c_i64(w.ws_len), H.ptr(w.counter), st)
    k2 = sorted(t(g, reps) for _ in range(3))[1]
    print(f"{tag:20s} n={n:9d} K4 {k4:7.2f} us ({12 * n / k4 / 1e3:5.0f} GB/s)   K2 {k2:6.2f} us ({4 * n / k2 / 1e3:5.0f} GB/s)", flush=True)
    del bufs
