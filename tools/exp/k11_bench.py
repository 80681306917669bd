"""K11 (torch-order mean, csrc/k_mean.hip) time per call at C5's layer sizes and reference
thread counts: event-timed groups of 20 calls through fakequant.torch_mean (3 kernels per
call: tiles, chunks, final), reported as read GB/s of the 4 B/elem pass."""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd  # noqa
from vsiquantization_amd.fakequant import torch_mean

dev = torch.device("cuda:0")
for n in (1_638_400, 6_553_600, 13_107_200, 52_428_800):
    xs = [torch.randn(n, device=dev) for _ in range(max(2, (512 << 20) // (4 * n)))]
    for threads in (1, 8, 16):
        for i in range(5):
            torch_mean(xs[i % len(xs)], act="relu", ref=(8, threads))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(20):
            torch_mean(xs[i % len(xs)], act="relu", ref=(8, threads))
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"n={n:>10d} threads={threads:>2d}  {us:8.2f} us/call  {4 * n / us / 1e3:7.0f} GB/s", flush=True)
