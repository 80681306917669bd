#!/usr/bin/env python3
"""Benchmark of the MI355X fake-quant hot path (BASELINE.json metric).

Default workload (config C2, the north-star kernel): per-channel asymmetric int8
MinMax observe + fake-quant FORWARD followed by the straight-through BACKWARD on
a 1024x1024x3x3 fp32 OIHW conv weight, one weight per step:

    fwd  vsiq_pc_observe_fq_f32   read W (4 B) + write Y (4 B) + write mask (1 B)   9 B/elem
    bwd  vsiq_ste_bwd_f32         read G (4 B) + read mask (1 B) + write dW (4 B)   9 B/elem

8 distinct (W, G, Y, mask, dW) slots (8 x 160 MB) rotate so no step is served from
the 256 MB Infinity Cache.  Launches go straight through the C ABI (the same entry
points the Python quantizers call), with precomputed arguments, on torch's current
stream.  HIP events bracket every kernel inside the timed region: their mean gives
each kernel's duration -> roofline.achieved.

  python bench.py [--gpus N --steps K --warmup W] [--workload c2|c3]

For N>1 (torchrun, one process per GPU) every rank processes its own weights (weak
scaling, no collective on this path); value = elements of all ranks / max time.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--workload", choices=["c2", "c3"], default="c2")
    p.add_argument("--slots", type=int, default=8)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    return p.parse_args()


# --------------------------------------------------------------------------- workloads
class C2PerChannel:
    """Per-channel asym int8 observe+fq fwd + STE bwd on a 1024x1024x3x3 weight."""

    name = "C2 per-channel asym int8 MinMax observe+fake-quant fwd + STE bwd"
    shape = (1024, 1024, 3, 3)
    qmin, qmax, sym = 0, 255, False

    def __init__(self, dev, slots, seed_base):
        from vsiquantization_amd import _hip as H
        from vsiquantization_amd.fakequant import qden
        self.H = H
        C = self.shape[0]
        self.n = n = 1
        for d in self.shape:
            self.n *= d
        n = self.n
        self.rowlen = n // C
        self.slots = []
        lib = H.lib()
        st = H.stream_of(dev)
        qd = qden(self.sym, 8, 1e-8)
        for i in range(slots):
            gen = torch.Generator(device=dev).manual_seed(seed_base + 2 * i)
            x = torch.randn(self.shape, device=dev, generator=gen) * 0.05
            gen.manual_seed(seed_base + 2 * i + 1)
            g = torch.randn(self.shape, device=dev, generator=gen)
            s = dict(x=x, g=g, y=torch.empty_like(x), gx=torch.empty_like(x),
                     mask=H.mask_buffer(C, self.n // C, dev),
                     rmin=torch.zeros(C, device=dev), rmax=torch.zeros(C, device=dev),
                     scale=torch.empty(C, dtype=torch.float64, device=dev),
                     zp=torch.empty(C, dtype=torch.float64, device=dev))
            P = {k: H.ptr(v) for k, v in s.items()}
            s["fwd"] = (P["x"], P["y"], None, P["mask"], H.c_i64(C), H.c_i64(self.rowlen), P["rmin"],
                        P["rmax"], P["scale"], P["zp"], None, 0, self.qmin, self.qmax, qd, 1e-8, st)
            s["bwd"] = (P["g"], P["mask"], P["gx"], H.c_i64(n), P["scale"], H.c_i64(self.rowlen), 0.0, st)
            self.slots.append(s)
        self.f_fwd = lib.vsiq_pc_observe_fq_f32
        self.f_bwd = lib.vsiq_ste_bwd_f32
        mbytes = 8 * int(lib.vsiq_mask_words(C, self.rowlen))   # 1 bit / element
        # algorithmic bytes per launch: fwd reads W, writes Y + mask bits; bwd reads G + mask bits,
        # writes dW (per-row qparams/state: 1024 x 24 B, negligible and not counted)
        self.kernels = {"pc_observe_fq_fwd": 8 * n + mbytes, "ste_bwd": 8 * n + mbytes}

    def launch(self, i):
        s = self.slots[i % len(self.slots)]
        return self.f_fwd(*s["fwd"]) | self.f_bwd(*s["bwd"])

    def launch_group(self, i0, cnt, ev):
        """cnt steps (slots i0..i0+cnt-1): all forwards, then all backwards (each slot's
        backward still follows its forward on the stream); events bracket each kernel run."""
        ns = len(self.slots)
        rc = 0
        ev[0].record()
        for j in range(cnt):
            rc |= self.f_fwd(*self.slots[(i0 + j) % ns]["fwd"])
        ev[1].record()
        for j in range(cnt):
            rc |= self.f_bwd(*self.slots[(i0 + j) % ns]["bwd"])
        ev[2].record()
        return rc

    def check(self):
        """Cheap self-check of slot 0 against the observer-free closed form (no oracle import)."""
        s = self.slots[0]
        x = s["x"].reshape(self.shape[0], -1)
        mn = torch.clamp(x.min(1).values, max=0.0).double().cpu()
        mx = torch.clamp(x.max(1).values, min=0.0).double().cpu()
        scale = (mx - mn) / (255 + 1e-8)   # host f64 division (torch-GPU would use a reciprocal)
        return bool(torch.equal(scale, s["scale"].cpu()))


class C3Lsq:
    """LSQ learnable symmetric int8 fwd + STE bwd on a 512x3x224x224 activation."""

    name = "C3 LSQ learnable-scale sym int8 fwd + STE/scale-grad bwd"
    shape = (512, 3, 224, 224)

    def __init__(self, dev, slots, seed_base):
        from vsiquantization_amd import _hip as H
        self.H = H
        n = 1
        for d in self.shape:
            n *= d
        self.n = n
        lib = H.lib()
        st = H.stream_of(dev)
        w = H.workspace(dev, n)
        self.ws = w
        self.slots = []
        for i in range(min(slots, 2)):   # 2 slots x 1.2 GB already defeat the MALL
            gen = torch.Generator(device=dev).manual_seed(seed_base + 2 * i)
            x = torch.randn(self.shape, device=dev, generator=gen)
            gen.manual_seed(seed_base + 2 * i + 1)
            g = torch.randn(self.shape, device=dev, generator=gen)
            s = dict(x=x, g=g, y=torch.empty_like(x), gx=torch.empty_like(x),
                     scale=torch.tensor(0.03, dtype=torch.float64, device=dev),
                     grads=torch.empty(2, dtype=torch.float64, device=dev))
            P = {k: H.ptr(v) for k, v in s.items()}
            gscale = (127 * n) ** -0.5
            s["fwd"] = (P["x"], P["y"], None, None, H.c_i64(n), None, P["scale"], 0.0, None, 0.0, 0, 0,
                        -128, 127, st)
            s["bwd"] = (P["g"], P["x"], P["gx"], H.c_i64(n), P["scale"], 0.0, None, 0.0, 0, -128, 127,
                        gscale, P["grads"], H.ptr(w.ws), H.c_i64(w.ws_len), H.ptr(w.counter), st)
            self.slots.append(s)
        self.f_fwd = lib.vsiq_fq_fwd_f32
        self.f_bwd = lib.vsiq_lsq_bwd_f32
        self.kernels = {"fq_fwd": 8 * n, "lsq_bwd": 12 * n}

    launch = C2PerChannel.launch
    launch_group = C2PerChannel.launch_group

    def check(self):
        return True


# --------------------------------------------------------------------------- CPU baseline
def cpu_baseline(workload, seconds):
    """The reference's eager-torch op sequence (oracle/eager_torch.py) on the host cores."""
    from oracle import eager_torch as E
    threads = max(1, min(16, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    gen = torch.Generator().manual_seed(0)
    if workload == "c2":
        rows = 64   # bounded sample: 64 of the 1024 out-channels (same row length 9216)
        w = torch.randn(rows, 1024, 3, 3, generator=gen) * 0.05
        g = torch.randn(rows, 1024, 3, 3, generator=gen)
        fn = lambda: E.per_channel_step(w, g, symmetric=False, bits=8)  # noqa: E731
        n = w.numel()
        sample = f"{rows} of 1024 out-channels of the 1024x1024x3x3 weight (9216 elem/row), fwd+bwd"
    else:
        x = torch.randn(64, 3, 224, 224, generator=gen)
        g = torch.randn(64, 3, 224, 224, generator=gen)
        fn = lambda: E.lsq_step(x, g)  # noqa: E731
        n = x.numel()
        sample = "64 of 512 images of the 512x3x224x224 activation, fwd+bwd"
    fn()
    best, t_end, iters = float("inf"), time.perf_counter() + seconds, 0
    while time.perf_counter() < t_end or iters < 2:
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
        iters += 1
    try:
        model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:  # noqa: BLE001
        model = platform.processor()
    return {"value": n / best / 1e6, "unit": "Melem/s", "cores": threads, "kind": "port",
            "sample": f"{sample}; min of {iters} runs; torch {torch.__version__} CPU, {model}, "
                      f"os.cpu_count()={os.cpu_count()}"}


# --------------------------------------------------------------------------- main
def load_pmc_traffic(workload, kernel):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        return d[workload][kernel]["hbm_bytes_per_launch"]
    except Exception:  # noqa: BLE001
        return None


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    import vsiquantization_amd  # noqa: F401  (torch first, then the HIP library)

    W = (C2PerChannel if a.workload == "c2" else C3Lsq)(dev, a.slots, 1000 * rank)
    for i in range(a.warmup):
        assert W.launch(i) == 0
    torch.cuda.synchronize()
    ok = W.check()

    ns = len(W.slots)
    groups = [(g0, min(ns, a.steps - g0)) for g0 in range(0, a.steps, ns)]
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in groups]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rc = 0
    for (g0, cnt), ev in zip(groups, evs):
        rc |= W.launch_group(g0, cnt, ev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    assert rc == 0, f"kernel launch failed rc={rc}"
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)

    names = list(W.kernels)
    dur = {names[0]: sum(e[0].elapsed_time(e[1]) for e in evs) / a.steps * 1e-3,
           names[1]: sum(e[1].elapsed_time(e[2]) for e in evs) / a.steps * 1e-3}
    dom = max(dur, key=dur.get)
    achieved = W.kernels[dom] / dur[dom] / 1e9
    traffic = load_pmc_traffic(a.workload, dom)
    per_kernel = {k: {"avg_us": dur[k] * 1e6, "alg_bytes": W.kernels[k],
                      "GBps": W.kernels[k] / dur[k] / 1e9,
                      "frac": W.kernels[k] / dur[k] / 1e9 / HBM_PEAK_GBS} for k in names}

    total_elems = W.n * a.steps * world
    out = {
        "metric": "Melements/s fake-quant fwd+bwd (per-channel int8) + achieved HBM GB/s vs roofline"
        if a.workload == "c2" else "Melements/s LSQ fake-quant fwd+bwd + achieved HBM GB/s vs roofline",
        "value": total_elems / dt / 1e6,
        "unit": "Melem/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (torch.randn, seeded per rank/slot)",
        "config": {"workload": W.name, "shape": list(W.shape), "elements_per_step": W.n,
                   "slots": len(W.slots), "parallelism": f"replicas x{world} (independent weights, "
                                                         "no collective on this path)",
                   "self_check": ok},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic},
        "kernels": per_kernel,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.workload, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
