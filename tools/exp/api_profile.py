"""torch.profiler view of the C2 step through the public API (host ops + kernels).
Experiment only."""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd as V  # noqa
dev = torch.device("cuda:0")
w = torch.randn(1024, 1024, 3, 3, device=dev) * 0.05
g = torch.randn_like(w)
q = V.PerChannelUniformQuantizer(8, False)


def step():
    wr = w.detach().requires_grad_(True)
    obs = V.PerChannelMinMaxObserver(False)
    y, _ = obs.observe_quantize(wr, q)
    y.backward(g)


for _ in range(20):
    step()
torch.cuda.synchronize()
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    for _ in range(20):
        step()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=40))
