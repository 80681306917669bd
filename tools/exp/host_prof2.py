"""cProfile of the host side of K1 / K4 wrapper calls on a tiny tensor (host-bound).
Experiment only."""
import cProfile, os, pstats, sys, time, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd as V  # noqa
from vsiquantization_amd import fakequant as FQ
dev = torch.device("cuda:0")
x = torch.randn(64, 64, device=dev)
g = torch.randn(64, 64, device=dev)
s = torch.nn.Parameter(torch.tensor(0.05, dtype=torch.float64, device=dev))
N = 5000


def bwd():
    FQ.lsq_backward(g, x, s, 0, -8, 7, 0.01, False)


def fwd():
    FQ.fake_quant(x, s, 0, -8, 7)


for name, fn in (("lsq_backward", bwd), ("fake_quant", fwd)):
    for _ in range(100):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(N):
        fn()
    torch.cuda.synchronize()
    print(f"{name:14s} {(time.perf_counter() - t) / N * 1e6:.2f} us/call", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(N):
        fn()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(12)
