"""The C2 step through the public Python API (PerChannelMinMaxObserver.observe_quantize +
backward) eager and graph-replayed, as bench.py reports it, plus torch's own x*1 fwd+bwd
on the same tensor for the host-speed reference of the box."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

dev = torch.device("cuda:0")
med, mn = bench.api_us_per_step(dev)
print(f"api_us_per_step median {med:.1f} min {mn:.1f}", flush=True)
print(f"api_graph_us_per_step {bench.api_graph_us_per_step(dev):.1f}", flush=True)
w = (torch.randn(1024, 1024, 3, 3, device=dev) * 0.05).requires_grad_(True)
g = torch.randn_like(w)
for _ in range(50):
    (w * 1.0).backward(g)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(300):
    w.grad = None
    (w * 1.0).backward(g)
torch.cuda.synchronize()
print(f"torch x*1 fwd+bwd {(time.perf_counter() - t0) / 300 * 1e6:.1f} us", flush=True)
