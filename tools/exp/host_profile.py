"""cProfile of the learnable fwd+bwd Python path (experiment only)."""
import cProfile, pstats, os, sys, time, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd as V
dev = "cuda:0"
x = torch.randn(64, 64, device=dev, requires_grad=True)
g = torch.randn(64, 64, device=dev)
q = V.UniformQuantizer(4, True)
s = torch.nn.Parameter(torch.tensor(0.05, dtype=torch.float64, device=dev))
def step():
    q.quantize(x, s, 0, True).backward(g)
for _ in range(50):
    step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(300):
    step()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
# without autograd: direct lsq_backward
from vsiquantization_amd import fakequant as FQ
xd = x.detach()
def bwd_only():
    FQ.lsq_backward(g, xd, s, 0, -8, 7, 1e-3, False)
for _ in range(50):
    bwd_only()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(1000):
    bwd_only()
torch.cuda.synchronize()
print("lsq_backward direct", (time.perf_counter() - t) * 1e3, "us/call")
