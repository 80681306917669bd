"""Host time per launch at C2 size (1024x1024x3x3), the GPU left to queue up: the host
loop's own duration (no sync inside), divided by the launches, median of 7 runs of 150.

  capi_auto / capi_fixed   vsiq_pc_observe_fq_f32 through ctypes, store gate tuned online
                           (the default) vs forced (VSIQ_TUNE_STORE_GATE: no tuner code)
  api_fwd_auto / _fixed    the public observe_quantize forward (bound C++ op)
  torch_fwd                x * 1.0 (grad-requiring x)
  api_step_auto / _fixed   observe_quantize + backward
  torch_step               (x * 1.0).backward(g)

usage: python tools/exp/launch_host.py"""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd as V  # noqa: E402
from vsiquantization_amd import _hip as H  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    lib = H.lib()
    st = H.stream_of(dev)
    shape = (1024, 1024, 3, 3)
    C, rowlen = 1024, 1024 * 9
    x = (torch.randn(shape, device=dev) * 0.05).requires_grad_(True)
    g = torch.randn(shape, device=dev)
    y = torch.empty_like(x)
    mask = torch.empty(int(lib.vsiq_mask_words(C, rowlen)), dtype=torch.int64, device=dev)
    rmin, rmax = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    sc, zp = torch.empty(C, dtype=torch.float64, device=dev), torch.empty(C, dtype=torch.float64, device=dev)
    obs, q = V.PerChannelMinMaxObserver(False), V.PerChannelUniformQuantizer(8, False)
    qd = 255.0

    def capi():
        lib.vsiq_pc_observe_fq_f32(H.ptr(x), H.ptr(y), None, H.ptr(mask), C, rowlen, H.ptr(rmin), H.ptr(rmax),
                                   H.ptr(sc), H.ptr(zp), None, 0, 0, 255, qd, 1e-8, st)

    def api_fwd():
        obs.observe_quantize(x, q)

    def torch_fwd():
        x * 1.0

    def api_step():
        x.grad = None
        yy, _ = obs.observe_quantize(x, q)
        yy.backward(g)

    def torch_step():
        x.grad = None
        (x * 1.0).backward(g)

    def host_us(fn, n=150):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        t = time.perf_counter() - t0
        torch.cuda.synchronize()
        return t / n * 1e6

    res = {}
    for r in range(8):
        for mode in ("auto", "fixed"):
            H.set_tuning(H.TUNE_STORE_GATE, -1 if mode == "auto" else 520)
            for name, fn in (("capi", capi), ("api_fwd", api_fwd), ("api_step", api_step)):
                v = host_us(fn)
                if r:
                    res.setdefault(f"{name}_{mode}", []).append(v)
        H.set_tuning(H.TUNE_STORE_GATE, -1)
        for name, fn in (("torch_fwd", torch_fwd), ("torch_step", torch_step)):
            v = host_us(fn)
            if r:
                res.setdefault(name, []).append(v)
    print(json.dumps({k: round(statistics.median(v), 2) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
