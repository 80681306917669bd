"""Host (Python) cost per quantizer call through the public API on small tensors, where
the kernels are microseconds: wall time per call with the GPU kept busy ahead.
Experiment only."""
import os, sys, time, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd as V
from vsiquantization_amd.quantizers.quantization_manager import QuantizationManager

dev = "cuda:0"
x = torch.randn(64, 64, device=dev, requires_grad=True)
g = torch.randn(64, 64, device=dev)


def wall(fn, reps=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


q = V.UniformQuantizer(4, True)
s = torch.nn.Parameter(torch.tensor(0.05, dtype=torch.float64, device=dev))
print(f"learnable fwd              {wall(lambda: q.quantize(x, s, 0, True)):7.1f} us/call", flush=True)
print(f"learnable fwd+bwd          {wall(lambda: q.quantize(x, s, 0, True).backward(g)):7.1f} us/call", flush=True)
print(f"fixed fwd (no grad)        {wall(lambda: q.quantize(x.detach(), 0.05, 0, False)):7.1f} us/call", flush=True)
qm = QuantizationManager("UniformQuantizer", "MinMaxObserver", 8, True, is_learning_scale=False)
qm.is_quantize = False
xd = x.detach()
print(f"manager observe (calib)    {wall(lambda: qm.quantize(xd)):7.1f} us/call", flush=True)
qm.dist_defer = True
print(f"manager observe (deferred) {wall(lambda: qm.quantize(xd), reps=500):7.1f} us/call", flush=True)
qm.dist_defer = False
qm._pending_records = []
qm.is_quantize = True
print(f"manager observe+quantize   {wall(lambda: qm.quantize(xd)):7.1f} us/call", flush=True)
t = torch.randn(64, 64, device=dev)
print(f"torch eager reference op chain (x/s+zp, round, clamp, sub, mul) {wall(lambda: (torch.clamp(torch.round(t / 0.05 + 0), -8, 7) - 0) * 0.05):7.1f} us/call", flush=True)


class _Id(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a):
        return a.clone()

    @staticmethod
    def backward(ctx, ga):
        return ga


print(f"trivial custom Function fwd+bwd {wall(lambda: _Id.apply(x).backward(g)):7.1f} us/call", flush=True)
sp = torch.nn.Parameter(torch.tensor(0.05, dtype=torch.float64, device=dev))


def ref_chain():
    ss = sp.float()
    y = (torch.clamp(torch.round(x / ss), -8, 7)) * ss
    y.backward(g)


print(f"torch eager learnable chain fwd+bwd {wall(ref_chain):7.1f} us/call", flush=True)
