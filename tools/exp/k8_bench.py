"""K8 (one-launch observe + fake quant of a small tensor) vs K2 + K1 across sizes.
Experiment only: back-to-back launches, events, median of 5."""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vsiquantization_amd import fakequant as FQ
dev = torch.device("cuda:0")


def t(fn, reps=200):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(20):
        fn()
    torch.cuda.synchronize(); s.record()
    for _ in range(reps):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for n in (432, 4608, 9216, 16384, 32768, 65536):
    x = torch.randn(n, device=dev)
    ra, rb = torch.zeros(2, device=dev), torch.zeros(2, device=dev)
    k8 = lambda: FQ.observe_fake_quant(x, symmetric=True, qmin=-128, qmax=127, run_minmax=ra)
    def k21():
        qp, _ = FQ.observe_tensor(x, symmetric=True, run_minmax=rb)
        FQ.fake_quant(x, None, None, -128, 127, qp=qp)
    a = sorted(t(k8) for _ in range(5))[2]
    b = sorted(t(k21) for _ in range(5))[2]
    print(f"n {n:6d}: K8 {a:6.2f} us   K2+K1 {b:6.2f} us", flush=True)
