"""Host cost of one launch (no sync), C2 shapes: where do the microseconds go?
ctypes overhead alone, the STE launch with the store-gate tuner on / off / forced,
torch's own elementwise launch, and a bare hipLaunchKernel of the same kernel through
the C ABI with the gate forced (no tuner bookkeeping).  Enqueue-only timing: the GPU
is kept busy behind a 20 ms sleep so the queue never drains."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import bench  # noqa: E402
from vsiquantization_amd import _hip as H  # noqa: E402


def enqueue_us(fn, n=200):
    best = []
    for _ in range(5):
        torch.cuda.synchronize()
        torch.cuda._sleep(40_000_000)
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        best.append((time.perf_counter() - t0) / n * 1e6)
        torch.cuda.synchronize()
    return sorted(best)[2]


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    W = bench.C2PerChannel(dev, 1, 0)
    for i in range(400):
        W.launch(i)
    torch.cuda.synchronize()
    lib = H.lib()
    s = W.slots[0]
    bwd, fwd = s["bwd"], s["fwd"]
    x, y = s["x"], s["y"]
    rows = [("ctypes call of vsiq_abi_version", lambda: lib.vsiq_abi_version()),
            ("STE launch, tuner on (tuned site)", lambda: lib.vsiq_ste_bwd_f32(*bwd)),
            ("K3 launch, tuner on (tuned site)", lambda: lib.vsiq_pc_observe_fq_f32(*fwd)),
            ("torch.mul(x, 1.0, out=y)", lambda: torch.mul(x, 1.0, out=y)),
            ("torch.empty_like(x)", lambda: torch.empty_like(x))]
    for name, fn in rows:
        print(f"{name:40s} {enqueue_us(fn):7.2f} us", flush=True)
    H.set_tuning(H.TUNE_STORE_GATE, 528)
    print(f"{'STE launch, gate forced (no tuner)':40s} {enqueue_us(lambda: lib.vsiq_ste_bwd_f32(*bwd)):7.2f} us")
    print(f"{'K3 launch, gate forced (no tuner)':40s} {enqueue_us(lambda: lib.vsiq_pc_observe_fq_f32(*fwd)):7.2f} us")
    H.set_tuning(H.TUNE_STORE_GATE, -1)
    ext = H.torch_ext()
    import vsiquantization_amd as V
    xg = s["x"].clone().requires_grad_(True)
    obs, q = V.PerChannelMinMaxObserver(False), V.PerChannelUniformQuantizer(8, False)
    print(f"{'observe_quantize fwd (C++ node)':40s} {enqueue_us(lambda: obs.observe_quantize(xg, q)):7.2f} us")
    yv, _ = obs.observe_quantize(xg, q)
    g = torch.randn_like(xg)

    def bwd_only():
        yy, _ = obs.observe_quantize(xg, q)
        xg.grad = None
        yy.backward(g)
    print(f"{'observe_quantize fwd + backward()':40s} {enqueue_us(bwd_only, n=100):7.2f} us")

    def trivial():
        xg.grad = None
        (xg * 1.0).backward(g)
    print(f"{'torch (x*1).backward(g)':40s} {enqueue_us(trivial, n=100):7.2f} us")


if __name__ == "__main__":
    main()
