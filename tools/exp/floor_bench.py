"""Per-launch floor for read-only kernels at C5 layer sizes: empty launch, a plain
float4 read (stream_kernels.so k_read, best grid) and K2p (vsiq_act_observe_part_f32).
Experiment only."""
import ctypes, os, sys, torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import vsiquantization_amd  # noqa
from vsiquantization_amd import _hip as H
from vsiquantization_amd.fakequant import part_slot_doubles
lib = ctypes.CDLL(os.path.join(HERE, "stream_kernels.so"))
dev = torch.device("cuda:0")
st = H.stream_of(dev)
P = ctypes.c_void_p
out = torch.zeros(1, device=dev)
for kv in os.environ.get("TUNE", "").split():
    k, v = kv.split("=")
    H.set_tuning(int(k), int(v))
TAG = os.environ.get("VSIQ_LIBRARY", "default")[-12:] + os.environ.get("TUNE", "")


def t(fn, reps=200):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(8):
        fn(i)
    torch.cuda.synchronize(); s.record()
    for i in range(reps):
        fn(i)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


print(f"empty launch (k_read n=0, grid 1)  {t(lambda i: lib.exp_read(P(out.data_ptr()), P(out.data_ptr()), ctypes.c_int64(0), 1, st)):6.2f} us")
for n in (1638400, 3276800, 6553600, 13107200, 26214400, 52428800):
    SL = max(2, min(16, (1600 << 20) // (4 * n)))
    xs = [torch.randn(n, device=dev) for _ in range(SL)]
    best = min((t(lambda i: lib.exp_read(P(xs[i % SL].data_ptr()), P(out.data_ptr()), ctypes.c_int64(n // 4), g, st)), g)
               for g in (256, 512, 1024, 2048, 4096))
    parts = torch.zeros(part_slot_doubles(n), dtype=torch.float64, device=dev)
    k2p = t(lambda i: H.lib().vsiq_act_observe_part_f32(P(xs[i % SL].data_ptr()), H.c_i64(n), 1, H.ptr(parts),
                                                        H.c_i64(parts.numel()), st))
    print(f"{TAG:24s} n={n:9d}  read {best[0]:6.2f} us (grid {best[1]}, {4 * n / best[0] / 1e3:5.0f} GB/s)   "
          f"K2p {k2p:6.2f} us ({4 * n / k2p / 1e3:5.0f} GB/s)", flush=True)
    del xs
