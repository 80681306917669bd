"""Delayed store phase vs tensor size (copy-shaped k_phase, SU=9, barrier). Experiment only."""
import ctypes, os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd  # noqa
HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "phase_exp.so"))
dev = torch.device("cuda:0")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = ctypes.c_void_p


def t(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(4):
        assert fn(i) == 0
    torch.cuda.synchronize(); s.record()
    for i in range(reps):
        fn(i)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for n in (1 << 20, 1600 * 1024, 9437184 // 2, 9437184, 2 * 9437184, 26 * 1 << 20, 77070336):
    sl = max(2, min(16, (600 << 20) // (8 * n)))
    xs = [torch.randn(n, device=dev) for _ in range(sl)]
    ys = [torch.empty(n, device=dev) for _ in range(sl)]
    reps = max(16, min(256, (4 << 30) // (8 * n)))
    for su, mode in ((2, 0), (9, 0), (9, 1), (9, 2)):
        row = []
        for slp in ((0,) if su == 2 else (0, 32, 64, 80, 96, 127)):
            v = sorted(t(lambda i: lib.exp_phase(P(xs[i % sl].data_ptr()), P(ys[i % sl].data_ptr()),
                                                  ctypes.c_int64(n), su, mode, slp, st), reps) for _ in range(3))[1]
            row.append(f"s{slp}:{v:7.2f}us/{8 * n / v / 1e3:5.0f}")
        print(f"n={n:9d} su{su} mode{mode}  " + "  ".join(row), flush=True)
    del xs, ys
