"""Host cost of the public-API C2 step on a SMALL weight (64x16x3x3: the kernels take ~3 us,
so every loop below is host-bound and measures host time per step), interleaved, median
of 7 runs of 2000 steps, us per step:

  ours_step      PerChannelMinMaxObserver.observe_quantize(x, q) + backward (the API step)
  torch_step     (x * 1.0).backward(g)                             (torch's trivial step)
  ours_fwd       observe_quantize only (graph built, not run backward)
  torch_fwd      x * 1.0 only
  op_fwd         the bound C++ op called directly (no Python checks)
  ours_fwd_ng    observe_quantize under no_grad (the non-autograd launch path)

usage: python tools/exp/api_host.py"""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd as V  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    shape = (64, 16, 3, 3)
    x = (torch.randn(shape, device=dev) * 0.05).requires_grad_(True)
    g = torch.randn(shape, device=dev)
    obs, q = V.PerChannelMinMaxObserver(False), V.PerChannelUniformQuantizer(8, False)
    obs.observe_quantize(x, q)
    op = obs._op[2]

    def ours_step():
        x.grad = None
        y, _ = obs.observe_quantize(x, q)
        y.backward(g)

    def torch_step():
        x.grad = None
        (x * 1.0).backward(g)

    def ours_fwd():
        obs.observe_quantize(x, q)

    def torch_fwd():
        x * 1.0

    def op_fwd():
        op(x)

    def ours_fwd_ng():
        with torch.no_grad():
            obs.observe_quantize(x, q)

    fns = dict(ours_step=ours_step, torch_step=torch_step, ours_fwd=ours_fwd, torch_fwd=torch_fwd,
               op_fwd=op_fwd, ours_fwd_ng=ours_fwd_ng)
    res = {k: [] for k in fns}
    for r in range(8):
        for k, f in fns.items():
            for _ in range(50):
                f()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(2000):
                f()
            torch.cuda.synchronize()
            if r:
                res[k].append((time.perf_counter() - t0) / 2000 * 1e6)
    out = {k: round(statistics.median(v), 2) for k, v in res.items()}
    out["ratio_step"] = round(out["ours_step"] / out["torch_step"], 3)
    print(json.dumps(out), flush=True)
    if os.environ.get("PROFILE"):
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(3000):
            ours_step()
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(14)


if __name__ == "__main__":
    main()
