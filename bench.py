#!/usr/bin/env python3
"""Benchmark of the MI355X fake-quant hot path (BASELINE.json metric).

Headline workload (config C2, the north-star kernel): per-channel asymmetric int8
MinMax observe + fake-quant FORWARD followed by the straight-through BACKWARD on
a 1024x1024x3x3 fp32 OIHW conv weight, one weight per step:

    fwd  vsiq_pc_observe_fq_f32   read W (4 B) + write Y (4 B) + write mask (1 bit)
    bwd  vsiq_ste_bwd_f32         read G (4 B) + read mask (1 bit) + write dW (4 B)

8 distinct (W, G, Y, mask, dW) slots (8 x 160 MB) rotate so no step is served from
the 256 MB Infinity Cache.  Launches go straight through the C ABI (the same entry
points the Python quantizers call), with precomputed arguments, on torch's current
stream.  HIP events bracket the kernels inside the timed region: their mean gives
each kernel's duration -> roofline.achieved.

The same JSON line carries, under "configs", the other BASELINE configs measured in
the same run (C1 per-tensor, C3 LSQ, C4 YOLOv8n backbone, C5 calibration) and
"batched_act_quant" (north_star's batched activation quant: per-call observe with the
RCCL exchange + fake quant over a 1024-image batch split across the ranks), plus
"api_us_per_step" (the C2 step through the public Python API), beside
"api_torch_ref_us_per_step" (torch's own (x * 1.0).backward(g) on the same tensor and
box) and the learnable per-call step "api_learn_us_per_step" beside torch's x * s
("api_learn_torch_xs_us_per_step").

  python bench.py [--gpus N --steps K --warmup W] [--workload c1..c5] [--extras LIST]

--gpus N > 1 without a torchrun environment: this process (which never touches the
GPU) starts `torch.distributed.run` with N ranks, one GPU each, RCCL, and exits with
its return code.  Under torchrun, WORLD_SIZE must equal --gpus.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
ACT_BATCH = 1024        # batched activation quant: images over all ranks
EXTRA_STEPS = {"c1": (200, 20), "c3": (100, 10), "c4": (30, 6), "c5": (100, 20), "act": (20, 4)}   # short legs read low (clock ramp)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--workload", choices=["c1", "c2", "c3", "c4", "c5", "act"], default="c2")
    p.add_argument("--extras", default=None,
                   help="comma list of extra configs in the same line (c1,c3,c4,c5,act; 'none'); "
                        "default: all of them for the c2 headline, none otherwise")
    p.add_argument("--batch", type=int, default=256, help="C4 batch (reference: 256)")
    p.add_argument("--bits-w", type=int, default=2, help="C4 weight bits (YAML default 2; SURVEY also w8)")
    p.add_argument("--bits-a", type=int, default=4, help="C4 activation bits (YAML default 4; SURVEY also a8)")
    p.add_argument("--per-call-grads", action="store_true",
                   help="C4: fold each activation scale gradient inside its K4 launch (round 1) instead of "
                        "records-only K4 + one fold launch (enable_deferred_qparam_grads)")
    p.add_argument("--asym", action="store_true",
                   help="C3: the asymmetric variant (uint8 [0, 255], learnable zero point 3.0: LSQQuantizer, "
                        "SURVEY §8d) instead of symmetric int8")
    p.add_argument("--slots", type=int, default=8)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-api", action="store_true", help="skip the public-API C2 timing")
    p.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU timing budget per config and thread count")
    p.add_argument("--master-port", type=int, default=0)
    p.add_argument("--dry-run", action="store_true",
                   help="launcher rehearsal without a GPU: ranks join a gloo group and report")
    p.add_argument("--gate-table", default=None, metavar="PATH",
                   help="start from a store-gate table saved by --save-gate-table and freeze the tuner "
                        "(no candidate or drift launches: reproducible kernel timing)")
    p.add_argument("--save-gate-table", default=None, metavar="PATH",
                   help="after the headline workload's gates have settled, save the table to PATH")
    p.add_argument("--markers", action="store_true",
                   help="launch vsiq_trace_marker right before / after each timed region (outside the "
                        "wall-clock window), so tools/timed_region_stats.py can cut a rocprofv3 kernel trace "
                        "to the timed launches")
    p.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                   help="experiments: vsiq_set_tuning(KEY, VALUE) before the workload is built "
                        "(keys: include/vsiq.h VSIQ_TUNE_*)")
    a = p.parse_args(argv)
    if a.extras is None:
        a.extras = "c1,c3,c4,c5,act" if a.workload == "c2" else ""
    a.extras = [e for e in a.extras.split(",") if e and e != "none"]
    bad = [e for e in a.extras if e not in EXTRA_STEPS]
    if bad:
        p.error(f"unknown --extras {bad}")
    return a


# --------------------------------------------------------------------------- launcher
def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a, argv) -> int:
    """N ranks under torch.distributed.run as a CHILD process (this process has not
    touched the GPU, and is not replaced: it waits and returns the child's code)."""
    port = a.master_port or free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    return subprocess.call(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))


# --------------------------------------------------------------------------- timing events
class HipEvent:
    """A HIP timing event created with hipEventDisableSystemFence (hip_runtime_api.h: for
    events "only being used to measure timing"; "on some AMD GPU devices this can improve
    the accuracy of timing measurements by avoiding the cost of cache writeback and
    invalidation, and the performance impact of those actions on the execution of following
    work").  torch.cuda.Event records with the default system-scope release, so every
    event between two launch phases wrote the L2 back and invalidated it in the middle of
    the timed region.  Same interface as torch.cuda.Event (record / elapsed_time) on the
    current stream.  VSIQ_BENCH_EVENTS=torch uses torch's events instead."""

    FLAG = 0x20000000   # hipEventDisableSystemFence
    _rt = None

    @classmethod
    def rt(cls):
        if cls._rt is None:
            rt = ctypes.CDLL("libamdhip64.so.7")   # torch's already-mapped HIP runtime
            rt.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            rt.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            rt.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
            rt.hipEventDestroy.argtypes = [ctypes.c_void_p]
            cls._rt = rt
        return cls._rt

    def __init__(self):
        self.h = ctypes.c_void_p()
        rc = self.rt().hipEventCreateWithFlags(ctypes.byref(self.h), self.FLAG)
        assert rc == 0, f"hipEventCreateWithFlags rc={rc}"

    def record(self, stream=None):
        st = (stream or torch.cuda.current_stream()).cuda_stream
        rc = self.rt().hipEventRecord(self.h, ctypes.c_void_p(st))
        assert rc == 0, f"hipEventRecord rc={rc}"

    def elapsed_time(self, end):
        ms = ctypes.c_float()
        rc = self.rt().hipEventElapsedTime(ctypes.byref(ms), self.h, end.h)
        assert rc == 0, f"hipEventElapsedTime rc={rc}"
        return ms.value

    def __del__(self):
        if self.h and self._rt is not None:
            self._rt.hipEventDestroy(self.h)
            self.h = ctypes.c_void_p()


def timing_event():
    if os.environ.get("VSIQ_BENCH_EVENTS", "hip") == "torch":
        return torch.cuda.Event(enable_timing=True)
    return HipEvent()


def timing_events_kind():
    return ("torch.cuda.Event (system-scope release)" if os.environ.get("VSIQ_BENCH_EVENTS", "hip") == "torch"
            else "HIP events with hipEventDisableSystemFence")


# --------------------------------------------------------------------------- workloads
class C2PerChannel:
    """Per-channel asym int8 observe+fq fwd + STE bwd on a 1024x1024x3x3 weight."""

    key = "c2"
    name = "C2 per-channel asym int8 MinMax observe+fake-quant fwd + STE bwd"
    shape = (1024, 1024, 3, 3)
    qmin, qmax, sym = 0, 255, False

    def __init__(self, dev, slots, seed_base):
        from vsiquantization_amd import _hip as H
        from vsiquantization_amd.fakequant import qden
        self.H = H
        C = self.shape[0]
        n = 1
        for d in self.shape:
            n *= d
        self.n = n
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

    group = property(lambda self: len(self.slots))

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

    def codes_variant(self, groups=25):
        """SURVEY §8d's second C2 figure: the forward with the uint8 codes emitted as well
        (9 B/elem + the mask bits), timed like the headline (groups of one launch per slot
        between HIP events, after the store-gate tuner has settled this launch site)."""
        H, C = self.H, self.shape[0]
        dev = self.slots[0]["x"].device
        codes = [torch.empty(self.shape, dtype=torch.uint8, device=dev) for _ in self.slots]
        args = [(s["fwd"][0], s["fwd"][1], H.ptr(c), *s["fwd"][3:]) for s, c in zip(self.slots, codes)]
        for k in range(4000):
            assert self.f_fwd(*args[k % len(args)]) == 0
            if k % 8 == 7:
                torch.cuda.synchronize()
                if H.gate_tuning_pending() == 0:
                    break
        evs = [(timing_event(), timing_event()) for _ in range(groups)]
        for e0, e1 in evs:
            e0.record()
            for a in args:
                assert self.f_fwd(*a) == 0
            e1.record()
        torch.cuda.synchronize()
        us = sum(e0.elapsed_time(e1) for e0, e1 in evs) / (groups * len(args)) * 1e3
        alg = self.kernels["pc_observe_fq_fwd"] + self.n
        ok = bool(torch.equal(codes[0].reshape(C, -1)[:, :4096].float(),
                              (self.slots[0]["y"].reshape(C, -1)[:, :4096].double()
                               / self.slots[0]["scale"][:, None] + self.slots[0]["zp"][:, None]).round().float()))
        return {"avg_us": us, "alg_bytes": alg, "GBps": alg / us / 1e3, "frac": alg / us / 1e3 / 8000.0,
                "codes_match_y": ok}

    def alt_kernels(self, groups=25):
        """SURVEY §8f2 at the north-star shape (not in the headline step): the LEARNABLE
        per-channel quantizer on this weight (LSQFakeQuantize / a learnable
        PerChannelUniformQuantizer on axis 0, lsq_module.py:96-175, 317-340) -- the forward
        with the rounded learned zero point (vsiq_pcm_fq_fwd_f32, 8 B/elem) and the K6
        backward with scale and zero point learned (vsiq_pcm_lsq_bwd_f32, reads x and g,
        writes dx: 12 B/elem), each timed like the headline: groups of one launch per slot
        between HIP events, after the store-gate tuner has settled the site."""
        if self.key != "c2":
            return {}
        H, C, n = self.H, self.shape[0], self.n
        lib = H.lib()
        dev = self.slots[0]["x"].device
        st = H.stream_of(dev)
        wsn = int(lib.vsiq_pcm_workspace_doubles(C, self.rowlen))
        ws = torch.empty(max(wsn, 2), dtype=torch.float64, device=dev)
        gsc = torch.empty(C, dtype=torch.float64, device=dev)
        gzp = torch.empty(C, dtype=torch.float64, device=dev)
        fwd, bwd = [], []
        for s in self.slots:
            P = {k: H.ptr(s[k]) for k in ("x", "y", "g", "gx", "scale", "zp")}
            fwd.append((P["x"], P["y"], None, None, H.c_i64(C), H.c_i64(self.rowlen), H.c_i64(C), P["scale"], P["zp"],
                        1, self.qmin, self.qmax, st))
            bwd.append((P["g"], P["x"], P["gx"], H.c_i64(C), H.c_i64(self.rowlen), H.c_i64(C), P["scale"], P["zp"], 1,
                        self.qmin, self.qmax, 1e-4, H.ptr(gsc), H.ptr(gzp), H.ptr(ws), H.c_i64(ws.numel()), st))
        out = {}
        for name, f, args, alg in (("pc_learn_fwd", lib.vsiq_pcm_fq_fwd_f32, fwd, 8 * n),
                                   ("pc_learn_bwd_k6", lib.vsiq_pcm_lsq_bwd_f32, bwd, 12 * n)):
            for k in range(4000):
                assert f(*args[k % len(args)]) == 0
                if k % 8 == 7:
                    torch.cuda.synchronize()
                    if H.gate_tuning_pending() == 0:
                        break
            evs = [(timing_event(), timing_event()) for _ in range(groups)]
            for e0, e1 in evs:
                e0.record()
                for a in args:
                    assert f(*a) == 0
                e1.record()
            torch.cuda.synchronize()
            us = sum(e0.elapsed_time(e1) for e0, e1 in evs) / (groups * len(args)) * 1e3
            out[name] = {"avg_us": us, "alg_bytes": alg, "GBps": alg / us / 1e3, "frac": alg / us / 1e3 / 8000.0,
                         "in_step": False}
        return out

    def check(self):
        """Slot 0, 64 rows spread over the tensor, against the reference's formulas restated
        in torch on the host (minmax.py:49-74 in float64, uniform.py:55,95 with IEEE fp32
        x / s, the STE gradient (g*s)/s): scale, zero point, y and dW bit-exact."""
        s = self.slots[0]
        C = self.shape[0]
        rows = torch.linspace(0, C - 1, 64).long()
        x = s["x"].reshape(C, -1)[rows].cpu()
        g = s["g"].reshape(C, -1)[rows].cpu()
        mn = torch.clamp(x.min(1).values, max=0.0).double()
        mx = torch.clamp(x.max(1).values, min=0.0).double()
        scale = (mx - mn) / (255 + 1e-8)
        zp = torch.round(-mn / (scale + 1e-8))
        s32, z32 = scale.float()[:, None], zp.float()[:, None]
        r = torch.round(x / s32 + z32)
        q = torch.clamp(r, 0, 255)
        y = (q - z32) * s32
        m = (r >= 0) & (r <= 255)
        gx = torch.where(m, (g * s32) / s32, torch.zeros_like(g))
        got = lambda k: s[k].reshape(C, -1)[rows].cpu()   # noqa: E731
        return bool(torch.equal(scale, s["scale"][rows].cpu()) and torch.equal(zp, s["zp"][rows].cpu())
                    and torch.equal(y.view(torch.int32), got("y").view(torch.int32))
                    and torch.equal(gx.view(torch.int32), got("gx").view(torch.int32)))


class C1PerTensor(C2PerChannel):
    """C1: the reference's minimal config -- MinMaxObserver + UniformQuantizer, per-tensor
    symmetric int8, on a 256x256 fp32 weight (observers/minmax.py:76-88 then
    quantizers/uniform.py:34-56): per step the per-call observe + fake quant the manager
    runs at this size, K9 (vsiq_act_observe_fq_parts_f32: K2p records, then one fake-quant
    launch whose every workgroup folds them into the running min/max + f64 qparams; no
    arrival chain); `C1_K10=1` times the one-launch K10 (vsiq_act_observe_fq_grid_f32: a
    grid barrier instead of the second launch; no faster), `C1_K2K1=1` round 1's
    K2 observe + K1 fake quant.
    65,536 elements: latency-bound (two launches), the GB/s are not the
    point."""

    key = "c1"
    name = "C1 per-tensor sym int8 MinMax observe + fake-quant fwd, 256x256"
    shape = (256, 256)

    def __init__(self, dev, slots, seed_base):
        from vsiquantization_amd import _hip as H
        from vsiquantization_amd.fakequant import qden
        self.H = H
        self.n = n = 256 * 256
        lib = H.lib()
        st = H.stream_of(dev)
        w = H.workspace(dev, n)
        qd = qden(True, 8, 1e-8)
        k10 = os.environ.get("C1_K10", "0") == "1"
        self.slots = []
        for i in range(slots):
            gen = torch.Generator(device=dev).manual_seed(seed_base + i)
            x = torch.randn(self.shape, device=dev, generator=gen)
            s = dict(x=x, y=torch.empty_like(x), rmm=torch.zeros(2, device=dev),
                     qp=torch.empty(H.QP_LEN, dtype=torch.float64, device=dev))
            P = {k: H.ptr(v) for k, v in s.items()}
            s["fwd"] = (P["x"], H.c_i64(n), None, P["rmm"], P["qp"], 1, qd, 1e-8, H.ptr(w.ws),
                        H.c_i64(w.ws_len), H.ptr(w.counter), st)
            s["bwd"] = (P["x"], P["y"], None, None, H.c_i64(n), P["qp"], None, 0.0, None, 0.0, 0, 0, -128, 127, st)
            self.slots.append(s)
            s["k9"] = (P["x"], P["y"], None, None, H.c_i64(n), 0, None, P["rmm"], P["qp"], 1, qd, 1e-8, -128, 127,
                       H.ptr(w.ws), H.c_i64(w.ws_len), st)
            if k10:
                s["k9"] = s["k9"][:-1] + (H.ptr(w.counter), st)
        self.f_fwd = lib.vsiq_observe_f32
        self.f_bwd = lib.vsiq_fq_fwd_f32
        self.f_k9 = lib.vsiq_act_observe_fq_grid_f32 if k10 else lib.vsiq_act_observe_fq_parts_f32
        self.k2k1 = os.environ.get("C1_K2K1", "0") == "1"
        # algorithmic bytes: observe reads x (4 B/elem), fake quant reads x, writes y (8);
        # K10 reads x once (registers across the grid barrier) and writes y: 8 B/elem
        self.kernels = ({"observe": 4 * n, "fq_fwd": 8 * n} if self.k2k1 else
                        {"observe_fq": (8 if k10 else 12) * n})

    def launch(self, i):
        if self.k2k1:
            return super().launch(i)
        return self.f_k9(*self.slots[i % len(self.slots)]["k9"])

    def launch_group(self, i0, cnt, ev):
        if self.k2k1:
            return super().launch_group(i0, cnt, ev)
        ns = len(self.slots)
        rc = 0
        ev[0].record()
        for j in range(cnt):
            rc |= self.f_k9(*self.slots[(i0 + j) % ns]["k9"])
        ev[1].record()
        return rc

    def check(self):
        """Slot 0 against the reference's formulas in torch on the host (IEEE fp32 x / s)."""
        s = self.slots[0]
        x = s["x"].cpu()
        mn, mx = min(0.0, float(x.min())), max(0.0, float(x.max()))
        scale = max(abs(mn), abs(mx)) / (2 ** 7 - 1 + 1e-8)
        want = torch.clamp(torch.round(x / scale), -128, 127) * scale
        return bool(torch.equal(s["y"].cpu().view(torch.int32), want.view(torch.int32)))


class C3Lsq(C2PerChannel):
    """LSQ learnable symmetric int8 fwd + STE bwd on a 512x3x224x224 activation."""

    key = "c3"
    name = "C3 LSQ learnable-scale sym int8 fwd + STE/scale-grad bwd"
    shape = (512, 3, 224, 224)
    scale0 = 0.03

    zp0 = 3.0

    def __init__(self, dev, slots, seed_base, asym=False):
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
        self.asym = asym
        self.qmin, self.qmax = (0, 255) if asym else (-128, 127)
        if asym:
            self.name = "C3 LSQ learnable-scale asym uint8 (learnable zero point 3.0) fwd + STE/scale/zp-grad bwd"
        self.gscale = (self.qmax * n) ** -0.5
        for i in range(min(slots, 2)):   # 2 slots x 1.2 GB already defeat the MALL
            gen = torch.Generator(device=dev).manual_seed(seed_base + 2 * i)
            x = torch.randn(self.shape, device=dev, generator=gen)
            gen.manual_seed(seed_base + 2 * i + 1)
            g = torch.randn(self.shape, device=dev, generator=gen)
            s = dict(x=x, g=g, y=torch.empty_like(x), gx=torch.empty_like(x),
                     scale=torch.tensor(self.scale0, dtype=torch.float64, device=dev),
                     zp=torch.tensor(self.zp0, dtype=torch.float64, device=dev),
                     grads=torch.empty(2, dtype=torch.float64, device=dev))
            P = {k: H.ptr(v) for k, v in s.items()}
            zp, za = (P["zp"], 1) if asym else (None, 0)   # zero_point_rounding (uniform.py:98-102)
            s["fwd"] = (P["x"], P["y"], None, None, H.c_i64(n), None, P["scale"], 0.0, zp, 0.0, za, 0,
                        self.qmin, self.qmax, st)
            s["bwd"] = (P["g"], P["x"], P["gx"], H.c_i64(n), P["scale"], 0.0, zp, 0.0, za, self.qmin, self.qmax,
                        self.gscale, P["grads"], H.ptr(w.ws), H.c_i64(w.ws_len), H.ptr(w.counter), st)
            self.slots.append(s)
        self.f_fwd = lib.vsiq_fq_fwd_f32
        self.f_bwd = lib.vsiq_lsq_bwd_f32
        self.kernels = {"fq_fwd": 8 * n, "lsq_bwd": 12 * n}

    def check(self):
        """Slot 0: y and grad_x bit-exact against the reference's formulas in torch on the
        host over the first 2M elements (uniform.py:55,95, IEEE fp32 x / s; STE (g*s)/s);
        the scale gradient within 1e-9 of the float64 sums of the reference's fp32
        autograd terms over the whole tensor (MulBackward g*(q - zp), DivBackward
        -(mask*g*s)*((x/s)/s), times gscale: SURVEY §8d's closed form)."""
        s = self.slots[0]
        k = 1 << 21
        s32 = torch.tensor(self.scale0, dtype=torch.float64).float()
        z32 = torch.tensor(self.zp0 if self.asym else 0.0, dtype=torch.float32)
        lo, hi = self.qmin, self.qmax
        acc, ok = 0.0, True
        for i0 in range(0, self.n, 1 << 23):
            x = s["x"].reshape(-1)[i0:i0 + (1 << 23)].cpu()
            g = s["g"].reshape(-1)[i0:i0 + (1 << 23)].cpu()
            r = torch.round(x / s32 + z32) if self.asym else torch.round(x / s32)
            q = torch.clamp(r, lo, hi)
            m = (r >= lo) & (r <= hi)
            gm = torch.where(m, g * s32, torch.zeros_like(g))
            acc += float((g * (q - z32)).double().sum()) + float(((-gm) * ((x / s32) / s32)).double().sum())
            if i0 == 0:
                y, gx = (q - z32) * s32, gm / s32
                ok = (torch.equal(y[:k].view(torch.int32), s["y"].reshape(-1)[:k].cpu().view(torch.int32))
                      and torch.equal(gx[:k].view(torch.int32), s["gx"].reshape(-1)[:k].cpu().view(torch.int32)))
        want = acc * self.gscale
        return bool(ok and abs(float(s["grads"][0]) - want) <= 1e-9 * abs(want))


def yolov8n_backbone(img=320, width=(3, 16, 32, 64, 128, 256), depth=(1, 2, 2)):
    """The 27 Conv(+BN+ReLU) layers of the reference's DarkNet backbone (nets/yolov8.py:75-117,
    yolo_v8_n widths/depths :224-227) in forward order: (cin, cout, k, stride, hout)."""
    layers, h = [], img

    def conv(cin, cout, k, s):
        nonlocal h
        h = (h + 2 * ((k - 1) // 2) - k) // s + 1
        layers.append((cin, cout, k, s, h))

    def csp(cin, cout, n):
        conv(cin, cout, 1, 1)
        for _ in range(n):
            conv(cout // 2, cout // 2, 3, 1)
            conv(cout // 2, cout // 2, 3, 1)
        conv((2 + n) * cout // 2, cout, 1, 1)

    conv(width[0], width[1], 3, 2)
    conv(width[1], width[2], 3, 2); csp(width[2], width[2], depth[0])
    conv(width[2], width[3], 3, 2); csp(width[3], width[3], depth[1])
    conv(width[3], width[4], 3, 2); csp(width[4], width[4], depth[2])
    conv(width[4], width[5], 3, 2); csp(width[5], width[5], depth[0])
    conv(width[5], width[5] // 2, 1, 1); conv(width[5] * 2, width[5], 1, 1)   # SPP
    return layers


def _act_ref(c, s32, qmin, qmax):
    """relu then the reference's fake quant (uniform.py:55,95), torch on the host."""
    a = torch.relu(c)
    return torch.clamp(torch.round(a / s32), qmin, qmax) * s32


class C4Backbone:
    """C4: the YOLOv8n backbone's 27 ConvBnReLU quantizers at 320x320, batch 256, in the
    learning phase: the 27 learnable weight fake quants as one multi-tensor launch each way
    (k_multi.hip, the path of enable_multi_tensor_weights) and per layer the fused ReLU +
    learnable activation fake quant (K5: K1-relu fwd, K4-relu bwd records-only + ONE fold of
    the 27 activation scale gradients at the end, the path of enable_deferred_qparam_grads;
    ``deferred=False``: K4 with its in-kernel fold per layer).  The conv itself is
    MIOpen and out of scope: synthetic conv outputs of the right shapes stand in for it."""

    key = "c4"
    name = "C4 YOLOv8n backbone ConvBnReLU fake-quant (weights + fused ReLU/act), learnable"
    group = 4

    def __init__(self, dev, slots, seed_base, batch=256, bits_w=2, bits_a=4, deferred=True):
        from vsiquantization_amd import _hip as H
        self.H = H
        lib = H.lib()
        st = H.stream_of(dev)
        self.deferred = deferred
        self.layers = yolov8n_backbone()
        self.shape = (batch, 3, 320, 320)
        qw = (-(2 ** (bits_w - 1)), 2 ** (bits_w - 1) - 1)
        qa = (-(2 ** (bits_a - 1)), 2 ** (bits_a - 1) - 1)
        self.qa = qa
        self.bits = (bits_w, bits_a)
        gen = torch.Generator(device=dev).manual_seed(seed_base)
        self.fwd, self.bwd, self.keep = [], [], []
        wdesc = []
        n_act = n_w = 0
        for cin, cout, k, s_, h in self.layers:
            w = torch.randn(cout, cin, k, k, device=dev, generator=gen) * (2.0 / (cin * k * k)) ** 0.5
            c = torch.randn(batch, cout, h, h, device=dev, generator=gen)
            g = torch.randn(batch, cout, h, h, device=dev, generator=gen)
            gw = torch.randn_like(w)
            t = dict(w=w, c=c, g=g, gw=gw, wq=torch.empty_like(w), y=torch.empty_like(c),
                     gc=torch.empty_like(c), gwx=torch.empty_like(w),
                     sw=torch.tensor(float(w.abs().mean()) * 2 / (qw[1] ** 0.5), dtype=torch.float64, device=dev),
                     sa=torch.tensor(2 * 0.8 / (qa[1] ** 0.5), dtype=torch.float64, device=dev),
                     grads_w=torch.empty(2, dtype=torch.float64, device=dev),
                     grads_a=torch.empty(2, dtype=torch.float64, device=dev))
            t["ws_a"] = torch.empty(lib.vsiq_workspace_doubles(c.numel()), dtype=torch.float64, device=dev)
            t["cnt_a"] = torch.zeros(H.COUNTER_WORDS, dtype=torch.int32, device=dev)
            P = {kk: H.ptr(v) for kk, v in t.items()}
            nw, na = w.numel(), c.numel()
            gsw, gsa = (qw[1] * nw) ** -0.5, (qa[1] * na) ** -0.5
            self.fwd.append((lib.vsiq_act_fq_fwd_f32, (P["c"], P["y"], None, None, H.c_i64(na), H.ACT_RELU,
                                                       None, P["sa"], 0.0, None, 0.0, 0, 0, qa[0], qa[1], st)))
            if deferred:   # records only; the 27 folds in one launch at the end (quantizers/deferred.py)
                t["nrec"] = int(lib.vsiq_lsq_part_records(H.c_i64(na)))
                t["rec_a"] = torch.empty(2 * t["nrec"], dtype=torch.float64, device=dev)
                self.bwd.append((lib.vsiq_act_lsq_bwd_part_f32, (P["g"], P["c"], P["gc"], H.c_i64(na), H.ACT_RELU,
                                                                 P["sa"], 0.0, None, 0.0, 0, qa[0], qa[1],
                                                                 H.ptr(t["rec_a"]), H.c_i64(t["rec_a"].numel()), st)))
                t["gsa"] = gsa
            else:
                self.bwd.append((lib.vsiq_act_lsq_bwd_f32, (P["g"], P["c"], P["gc"], H.c_i64(na), H.ACT_RELU,
                                                            P["sa"], 0.0, None, 0.0, 0, qa[0], qa[1], gsa,
                                                            P["grads_a"], P["ws_a"], H.c_i64(t["ws_a"].numel()),
                                                            P["cnt_a"], st)))
            wdesc.append(dict(x=w.data_ptr(), y=t["wq"].data_ptr(), g=gw.data_ptr(), gx=t["gwx"].data_ptr(),
                              scale_dev=t["sw"].data_ptr(), grad_out=t["grads_w"].data_ptr(), n=nw,
                              gscale=gsw, qmin=qw[0], qmax=qw[1]))
            self.keep.append(t)
            n_act += na
            n_w += nw
        # the 27 weight quantizers: ONE multi-tensor launch each way (quantizers/foreach.py,
        # enable_multi_tensor_weights): all weight fake quants before the first conv, all
        # weight backwards once autograd has every weight gradient
        import ctypes
        self.wdesc = (H.LsqTensor * len(wdesc))()
        for i, d in enumerate(wdesc):
            for k, v in d.items():
                setattr(self.wdesc[i], k, v)
        wp = ctypes.cast(self.wdesc, ctypes.c_void_p)
        need = int(lib.vsiq_lsq_multi_workspace_doubles(wp, len(wdesc)))
        self.ws_w = torch.empty(max(need, 1), dtype=torch.float64, device=dev)
        self.cnt_w = torch.zeros(H.COUNTER_WORDS, dtype=torch.int32, device=dev)
        self.fwd.insert(0, (lib.vsiq_lsq_fwd_multi_f32, (wp, len(wdesc), st)))
        self.bwd.append((lib.vsiq_lsq_bwd_multi_f32, (wp, len(wdesc), H.ptr(self.ws_w), H.c_i64(self.ws_w.numel()),
                                                      H.ptr(self.cnt_w), st)))
        if deferred:   # autograd reaches the qparam bundle last: ONE fold of the 27 activation calls
            self.folds = (H.LsqFold * len(self.keep))()
            for i, t in enumerate(self.keep):
                self.folds[i] = H.LsqFold(t["rec_a"].data_ptr(), t["nrec"], None, 0.0, t["gsa"],
                                          t["grads_a"].data_ptr(), qa[0], qa[1], 0, 0)
            self.bwd.append((lib.vsiq_lsq_fold_multi, (ctypes.cast(self.folds, ctypes.c_void_p), len(self.keep), st)))
        self.n = n_act + n_w
        self.n_act, self.n_w = n_act, n_w
        self.slots = [None]
        # algorithmic bytes per step: fwd 8 B/elem (weights and activations; the fused ReLU 0),
        # bwd 12 B/elem (read g, read x or c, write grad)
        self.kernels = {"fwd_all_layers": 8 * self.n, "bwd_all_layers": 12 * self.n}

    def launch(self, i):
        rc = 0
        for f, a in self.fwd:
            rc |= f(*a)
        for f, a in self.bwd:
            rc |= f(*a)
        return rc

    def launch_group(self, i0, cnt, ev):
        rc = 0
        ev[0].record()
        for _ in range(cnt):
            for f, a in self.fwd:
                rc |= f(*a)
        ev[1].record()
        for _ in range(cnt):
            for f, a in self.bwd:
                rc |= f(*a)
        ev[2].record()
        return rc

    def check(self):
        """Layer 0 (the largest activation): the fused ReLU + act fake quant y bit-exact
        against torch on the host over the first 2M elements; grad zero where the conv
        output is negative (ReLU backward); every gradient record finite."""
        t = self.keep[0]
        k = 1 << 21
        c = t["c"].reshape(-1)[:k].cpu()
        s32 = t["sa"].cpu().float()
        y = _act_ref(c, s32, *self.qa)
        ok = torch.equal(y.view(torch.int32), t["y"].reshape(-1)[:k].cpu().view(torch.int32))
        neg = t["c"] < 0
        return bool(ok and (t["gc"][neg] == 0).all()
                    and all(bool(torch.isfinite(x["grads_a"]).all() and torch.isfinite(x["grads_w"]).all())
                            for x in self.keep))


class C5Calibration:
    """C5: calibration of the YOLOv8n backbone's 27 activation quantizers (MinMaxObserver,
    sym) on batches of 128 images per GPU (1024 over 8 GPUs), as calibrate_qat_model runs
    it by default (utils/quantize_manager.py:4-31 -> modules/fused.py:124-134 ->
    quantizers/fake_quantize.py:49-50; here QuantizationManager._observe_deferred_act): per
    batch and layer ONE K2o launch (vsiq_act_observe_part_out_f32) that reads the conv
    output c, writes y = relu(c) -- the tensor the next layer consumes -- and stores the
    deferred observer's partial records of relu(c) in its own device slot (8 B/elem: read
    4 + write 4; no fold, no atomics, no sync); after the last batch ONE deferred sync --
    one fold launch over all slots of all layers and batches, two RCCL all-reduces over the
    records, and the exact replay of every layer's running min/max (distributed.
    sync_calibration).  Driven through the C ABI so the Python manager's per-call host
    cost is not what is measured.  min/max are bit-identical to a 1-GPU run
    (tests/test_dist_gloo.py).  Synthetic conv outputs stand in for the conv (MIOpen, out
    of scope).

    `alt_kernels` times, on the same inputs, the opt-in observe-only multi-tensor pass
    (K2m, VSIQ_OBSERVE_BATCH=1: 27 layers' records in one launch, 4 B/elem, the activation
    not written) that round 2's C5 line measured."""

    key = "c5"
    name = "C5 YOLOv8n backbone calibration: per-layer fused-ReLU K2o (act out + observer records), deferred RCCL sync"
    group = 16

    def __init__(self, dev, slots, seed_base, batch=128, steps=16):
        from vsiquantization_amd import _hip as H
        from vsiquantization_amd.fakequant import part_out_slot_doubles, part_slot_doubles
        self.H = H
        lib = H.lib()
        self.st = H.stream_of(dev)
        self.layers = yolov8n_backbone()
        self.shape = (batch, 3, 320, 320)
        gen = torch.Generator(device=dev).manual_seed(seed_base)
        self.acts = [torch.randn(batch, co, h, h, device=dev, generator=gen) for _, co, _, _, h in self.layers]
        self.ys = [torch.empty_like(a) for a in self.acts]   # relu(c), what the next conv reads
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.steps = steps
        L = len(self.layers)
        self.stride = max(part_out_slot_doubles(a.numel()) for a in self.acts)
        self.parts = torch.zeros(steps, L, self.stride, dtype=torch.float64, device=dev)
        self.f_k2o = lib.vsiq_act_observe_part_out_f32
        self.args = [[(H.ptr(a), H.ptr(y), H.c_i64(a.numel()), H.ACT_RELU, self.parts[k, j].data_ptr(),
                       H.c_i64(self.stride), self.st) for j, (a, y) in enumerate(zip(self.acts, self.ys))]
                     for k in range(steps)]
        # K2m (alt_kernels): one observe-only multi-tensor launch per batch
        self.m_stride = max(part_slot_doubles(a.numel()) for a in self.acts)
        self.m_parts = torch.zeros(L, self.m_stride, dtype=torch.float64, device=dev)
        arr = (H.PartTensor * L)()
        for j, a in enumerate(self.acts):
            arr[j] = H.PartTensor(a.data_ptr(), a.numel(), self.m_parts[j].data_ptr(), self.m_stride)
        self.m_desc, self.f_k2m = arr, lib.vsiq_act_observe_part_multi_f32
        self.n = sum(a.numel() for a in self.acts)
        self.slots = [None]
        self.kernels = {"act_observe_out_all_layers": 8 * self.n, "sync": 0}
        self.minmax = None

    def _observe(self, step):
        """One calibration batch: the 27 layers' K2o launches, in layer order."""
        rc = 0
        f = self.f_k2o
        for args in self.args[step % self.steps]:
            rc |= f(*args)
        return rc

    def launch(self, i):
        """One (untimed, warmup) calibration batch, followed by the deferred sync over the
        batches so far, so that the timed region finds the fold / replay path warm too."""
        rc = self._observe(i)
        self._sync(min(self.steps, i + 1))
        return rc

    def _sync(self, k):
        """The deferred sync over the first k batches: one fold launch over every slot,
        all-reduce, running-state replay."""
        from vsiquantization_amd.distributed import allreduce_stats, replay_minmax_tensor
        from vsiquantization_amd.fakequant import fold_parts
        L = len(self.layers)
        recs = fold_parts(self.parts[:k].reshape(k * L, self.stride))
        recs = recs.reshape(k, L, -1).transpose(0, 1).contiguous()   # [layers, calls, ST_LEN]
        if self.world > 1:
            allreduce_stats(recs)
        self.minmax = replay_minmax_tensor(0.0, 0.0, recs)         # stays on the device
        self.recs = recs

    def launch_group(self, i0, cnt, ev):
        rc = 0
        ev[0].record()
        for j in range(cnt):
            rc |= self._observe(i0 + j)
        ev[1].record()
        self._sync(min(self.steps, i0 + cnt))
        ev[2].record()
        return rc

    def alt_kernels(self, reps=20):
        """The opt-in K2m pass (observe only, 4 B/elem) over the same 27 tensors, event-
        timed: {name: {avg_us, alg_bytes, GBps, frac}} (not part of the step)."""
        for _ in range(3):
            assert self.f_k2m(self.m_desc, len(self.acts), self.H.ACT_RELU, self.st) == 0
        e0, e1 = timing_event(), timing_event()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            assert self.f_k2m(self.m_desc, len(self.acts), self.H.ACT_RELU, self.st) == 0
        e1.record()
        torch.cuda.synchronize()
        dt = e0.elapsed_time(e1) * 1e-3 / reps
        b = 4 * self.n
        return {"observe_all_layers_k2m_opt_in": {"avg_us": dt * 1e6, "alg_bytes": b, "GBps": b / dt / 1e9,
                                                  "frac": b / dt / 1e9 / HBM_PEAK_GBS, "in_step": False,
                                                  "note": "VSIQ_OBSERVE_BATCH=1 path: observe only, the "
                                                          "activation not written"}}

    def check(self):
        """Running min/max after the sync identical on every rank; on one GPU equal to a
        direct reduction of relu(conv output), mean|x| within 1e-6 of torch's, and the
        written activations y == relu(c) bit for bit."""
        self._sync(1)
        mm = torch.stack(self.minmax, dim=-1)
        y_ok = all(torch.equal(y.view(torch.int32), torch.where(a < 0, torch.zeros_like(a), a).view(torch.int32))
                   for a, y in zip(self.acts[::9], self.ys[::9]))   # the CPU relu's bits (-0.0 kept)
        if self.world > 1:
            hi, lo = mm.clone(), mm.clone()
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            return bool(torch.equal(hi, lo)) and y_ok
        ref = [(min(0.0, float(torch.relu(a).min())), max(0.0, float(torch.relu(a).max()))) for a in self.acts]
        from vsiquantization_amd import _hip as H
        ma = [float(torch.relu(a).double().abs().mean()) for a in self.acts]
        got = self.recs[:, 0, H.ST_SUMABS] / self.recs[:, 0, H.ST_N]
        close = all(abs(float(v) - w) <= 1e-6 * w for v, w in zip(got, ma))
        return [tuple(r) for r in mm.tolist()] == ref and close and y_ok


class ActQuant:
    """north_star's batched activation quant: the YOLOv8n backbone's 27 activation
    quantizers in observe + quantize mode (calibrate, then
    activate_quantizer without learnable qparams) over a batch of 1024 images split
    across the ranks (1024/N per GPU: strong scaling).  Per layer and call: K2 observe
    of relu(conv output) (4 B/elem) -> K1 fused-ReLU fake quant reading the qparams by
    pointer (8 B/elem); with N > 1, between them one RCCL all_gather of the 10-double stats
    records, folded (rank order, running update, f64 qparams) inside the fake-quant launch
    (vsiq_act_fq_fwd_ranks_f32; QuantizationManager.dist_group,
    distributed.observe_gather_fake_quant).  Symmetric, observer 8-bit, quantizer
    4-bit (the YAML default a4 and the observer quirk)."""

    key = "act"
    name = "batched activation quant: YOLOv8n backbone, per-call MinMax observe (+RCCL) + fake quant, fused ReLU"
    group = 2

    def __init__(self, dev, world, rank, total_batch=ACT_BATCH, bits=4, exchange=None):
        """exchange: the per-call RCCL exchange (all_gather + K1r); default world > 1 (a
        1-rank group can force it to rehearse the collective path, tests)."""
        from vsiquantization_amd import _hip as H
        from vsiquantization_amd.fakequant import qden
        if total_batch % world:
            raise ValueError(f"batch {total_batch} does not split over {world} ranks")
        self.H = H
        lib = H.lib()
        st = H.stream_of(dev)
        self.world = world
        self.exchange = world > 1 if exchange is None else bool(exchange)
        self.batch = total_batch // world
        self.layers = yolov8n_backbone()
        self.shape = (self.batch, 3, 320, 320)
        self.qmin, self.qmax = -(2 ** (bits - 1)), 2 ** (bits - 1) - 1
        gen = torch.Generator(device=dev).manual_seed(7000 + rank)
        qd = qden(True, 8, 1e-8)
        self.L = []
        for _, co, _, _, h in self.layers:
            x = torch.randn(self.batch, co, h, h, device=dev, generator=gen)
            t = dict(x=x, y=torch.empty_like(x), rmm=torch.zeros(2, device=dev),
                     st=torch.empty(H.ST_LEN, dtype=torch.float64, device=dev),
                     qp=torch.empty(H.QP_LEN, dtype=torch.float64, device=dev))
            t["ws"] = torch.empty(lib.vsiq_workspace_doubles(x.numel()), dtype=torch.float64, device=dev)
            t["cnt"] = torch.zeros(H.COUNTER_WORDS, dtype=torch.int32, device=dev)
            P = {k: H.ptr(v) for k, v in t.items()}
            n = H.c_i64(x.numel())
            loc = not self.exchange   # no exchange: the observer pass updates the state and writes qparams itself
            t["obs"] = (P["x"], n, H.ACT_RELU, P["st"], P["rmm"] if loc else None, P["qp"] if loc else None,
                        1, qd, 1e-8, P["ws"], H.c_i64(t["ws"].numel()), P["cnt"], st)
            t["gat"] = torch.empty(world * H.ST_LEN, dtype=torch.float64, device=dev)
            t["fq"] = (P["x"], P["y"], None, None, n, H.ACT_RELU, P["qp"], None, 0.0, None, 0.0, 0, 0,
                       self.qmin, self.qmax, st)
            # N > 1: the gathered records folded inside the fake-quant launch (K1r)
            t["rfq"] = (P["x"], P["y"], None, None, n, H.ACT_RELU, H.ptr(t["gat"]), world, P["st"], P["rmm"],
                        P["qp"], 1, qd, 1e-8, self.qmin, self.qmax, st)
            self.L.append(t)
        self.f_obs, self.f_fq, self.f_rfq = (lib.vsiq_act_observe_f32, lib.vsiq_act_fq_fwd_f32,
                                             lib.vsiq_act_fq_fwd_ranks_f32)
        self.n = sum(t["x"].numel() for t in self.L)
        self.slots = [None]
        self.kernels = {"observe_quant_all_layers": 12 * self.n}

    def launch(self, i):
        rc = 0
        if not self.exchange:
            for t in self.L:
                rc |= self.f_obs(*t["obs"])
                rc |= self.f_fq(*t["fq"])
            return rc
        from vsiquantization_amd.distributed import collective_group
        grp = collective_group(None)   # under a HIP-graph capture: the world's capture-only twin
        for t in self.L:   # local K2 pass, ONE all_gather of the 10-double records, ONE fold + fq launch
            rc |= self.f_obs(*t["obs"])
            dist.all_gather_into_tensor(t["gat"], t["st"], group=grp)
            rc |= self.f_rfq(*t["rfq"])
        return rc

    def launch_group(self, i0, cnt, ev):
        rc = 0
        ev[0].record()
        for j in range(cnt):
            rc |= self.launch(i0 + j)
        ev[1].record()
        return rc

    def check(self):
        """qparams identical on every rank; layer 0's y bit-exact (first 2M elements)
        against torch on the host with the scale from the global max of relu(x)."""
        qp = torch.stack([t["qp"] for t in self.L])
        if self.world > 1:
            hi, lo = qp.clone(), qp.clone()
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            same = bool(torch.equal(hi, lo))
        else:
            same = True
        t = self.L[0]
        mx = t["x"].max().clamp_min(0.0).reshape(1)
        if self.world > 1:
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        s32 = torch.tensor(float(mx) / (127 + 1e-8)).float()
        k = 1 << 21
        y = _act_ref(t["x"].reshape(-1)[:k].cpu(), s32, self.qmin, self.qmax)
        return same and bool(torch.equal(y.view(torch.int32), t["y"].reshape(-1)[:k].cpu().view(torch.int32)))


# --------------------------------------------------------------------------- CPU baseline (§8d)
def cpu_thread_counts():
    """[os.cpu_count(), the CPUs this process may actually use (affinity and cgroup
    quota), OMP_NUM_THREADS] without duplicates: SURVEY §8d asks for os.cpu_count();
    on a shared GPU box the usable share can be far smaller, so both are timed."""
    total = os.cpu_count() or 1
    usable = total
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            usable = min(usable, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    out = [total]
    for c in (usable, int(os.environ.get("OMP_NUM_THREADS", "0") or 0)):
        if c and c not in out:
            out.append(c)
    return out, total, usable


def cpu_workload(workload, bits=(2, 4), frac=1):
    """(fn, elements, description): the workload as the reference's eager op sequence
    (oracle/eager_torch.py) on the host -- the WHOLE workload at frac=1, 1/frac of its
    out-channels / images for the thread-count probe."""
    from oracle import eager_torch as E
    gen = torch.Generator().manual_seed(0)
    if workload == "c1":
        from oracle.fakequant_np import minmax_qparams
        x = torch.randn(256, 256, generator=gen)

        def fn():   # observers/minmax.py:76-88 (two .item()) then uniform.py:54-55,95
            mn, mx = E.observe(x)
            s, z = minmax_qparams(mn, mx, True, 8)
            return E.fake_quant(x, s, z, -128, 127)
        return fn, x.numel(), "the whole 256x256 workload (observe + fake quant per call)"
    if workload == "c2":
        rows = 1024 // frac
        w = torch.randn(rows, 1024, 3, 3, generator=gen) * 0.05
        g = torch.randn(rows, 1024, 3, 3, generator=gen)
        return ((lambda: E.per_channel_step(w, g, symmetric=False, bits=8)), w.numel(),
                f"{rows} of the 1024 out-channels of the 1024x1024x3x3 weight, reference classes looped "
                "over the out-channels, fwd+bwd")
    if workload in ("c3", "c3asym"):
        imgs = 512 // frac
        x = torch.randn(imgs, 3, 224, 224, generator=gen)
        g = torch.randn(imgs, 3, 224, 224, generator=gen)
        zp = C3Lsq.zp0 if workload == "c3asym" else None
        return ((lambda: E.lsq_step(x, g, zero_point=zp)), x.numel(),
                f"{imgs} of the 512 images of the 512x3x224x224 activation, fwd+bwd"
                + (" (asymmetric, learnable zero point)" if zp is not None else ""))
    if workload == "c5":
        imgs = 128 // frac
        acts = [torch.randn(imgs, co, h, h, generator=gen) for _, co, _, _, h in yolov8n_backbone()]

        def fn():   # reference calibration per layer: relu, observer (2 .item()), 3 stats
            for c in acts:
                a = torch.relu(c)
                E.observe(a)
                a.abs().mean().item(), a.mean().item(), a.std().item()
        return (fn, sum(t.numel() for t in acts),
                f"{imgs} of the 128 images per GPU of one calibration batch through all 27 observers")
    if workload == "c4":
        imgs = 256 // frac
        tens = []
        for cin, cout, k, _, h in yolov8n_backbone():
            tens.append((torch.randn(cout, cin, k, k, generator=gen) * (2.0 / (cin * k * k)) ** 0.5,
                         torch.randn(cout, cin, k, k, generator=gen),
                         torch.randn(imgs, cout, h, h, generator=gen),
                         torch.randn(imgs, cout, h, h, generator=gen)))

        def fn():
            for w, gw, c, g in tens:
                E.lsq_step(w, gw, scale=0.05, bits=bits[0])
                E.lsq_step(c, g, scale=0.5, bits=bits[1], act="relu")
        return (fn, sum(t[0].numel() + t[2].numel() for t in tens),
                f"{imgs} of the 256 images through all 27 backbone layers (+ weights), w{bits[0]}/a{bits[1]}, fwd+bwd")
    if workload == "act":
        from oracle.fakequant_np import minmax_qparams
        imgs = 1024 // (64 * frac)
        acts = [torch.randn(imgs, co, h, h, generator=gen) for _, co, _, _, h in yolov8n_backbone()]

        def fn():   # per layer: relu, observer (2 .item()), 3 stats, qparams, fake quant (qm.py:55-90)
            for c in acts:
                a = torch.relu(c)
                mn, mx = E.observe(a)
                a.abs().mean().item(), a.mean().item(), a.std().item()
                s, z = minmax_qparams(mn, mx, True, 8)
                E.fake_quant(a, s, z, -8, 7)
        return (fn, sum(t.numel() for t in acts),
                f"{imgs} of the 1024 images through all 27 activation quantizers (observe + quantize per call)")
    raise ValueError(workload)


def _best_time(fn, seconds, max_runs=50):
    """min wall time of fn over >= 1 timed runs after one warm-up run, within ~seconds."""
    t0 = time.perf_counter()
    fn()
    t_end = time.perf_counter() + max(seconds - (time.perf_counter() - t0), 0.0)
    best, iters = float("inf"), 0
    while iters < 1 or (time.perf_counter() < t_end and iters < max_runs):
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
        iters += 1
    return best, iters


_THREAD_PLAN = None


def thread_plan(seconds=2.0):
    """Thread counts worth timing the whole workloads at: every count of
    cpu_thread_counts() (os.cpu_count() first) is probed once on the C1 op sequence
    (256x256 observe + fake quant: ~10 OpenMP regions); counts whose probe rate is below
    half of the best are not used for the whole workloads (on a GPU box whose usable CPU
    share is a fraction of os.cpu_count(), oversubscribed OpenMP regions run ~1000x
    slower and one whole workload would take minutes).  Returns (counts kept, probe
    rates Melem/s by count, os.cpu_count(), usable CPUs)."""
    global _THREAD_PLAN
    if _THREAD_PLAN is None:
        counts, total, usable = cpu_thread_counts()
        fn, n, _ = cpu_workload("c1")
        prev = torch.get_num_threads()
        probe = {}
        for th in counts:
            progress(f"cpu baseline: thread probe at {th} threads")
            torch.set_num_threads(th)
            probe[th] = n / _best_time(fn, seconds, max_runs=20)[0] / 1e6
        torch.set_num_threads(prev)
        best = max(probe.values())
        _THREAD_PLAN = ([th for th in counts if 2 * probe[th] >= best], probe, total, usable)
    return _THREAD_PLAN


def cpu_baseline(workload, seconds, bits=(2, 4)):
    """The reference's eager-torch op sequence on the host cores: the WHOLE
    workload (C4: 64 of its 256 images), min of N wall times after a warm-up run (within `seconds`, at least one
    timed run), at each thread count thread_plan() keeps (os.cpu_count() and the usable
    CPU count are both probed and recorded); value = the best whole-workload rate."""
    counts, probe, total, usable = thread_plan()
    # C4's whole workload (547M elements fwd + bwd) takes ~5 s per run on 16 host CPUs, so
    # a `seconds` budget held one timed run; a quarter of its images (same per-element
    # work) gives min-of-several like the other configs
    frac = 4 if workload == "c4" else 1
    fn, n, desc = cpu_workload(workload, bits, frac=frac)
    what = "whole workload" if frac == 1 else f"1/{frac} sample of the workload"
    prev = torch.get_num_threads()
    tried, runs = {}, {}
    for th in counts:
        progress(f"cpu baseline {workload}: {what} at {th} threads")
        torch.set_num_threads(th)
        t, runs[th] = _best_time(fn, seconds)
        tried[th] = n / t / 1e6
    torch.set_num_threads(prev)
    th = max(tried, key=tried.get)
    try:
        model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:  # noqa: BLE001
        model = platform.processor()
    out = {"value": tried[th], "unit": "Melem/s", "cores": int(th), "kind": "port",
           "sample": f"{desc}; min of {runs[th]} runs at {th} threads; torch {torch.__version__} CPU, {model}",
           "threads_whole": {str(k): v for k, v in tried.items()},
           "thread_probe_c1": {str(k): v for k, v in probe.items()},
           "os_cpu_count": total, "usable_cpus": usable, "cpu_model": model}
    if workload == "c1":
        out["product_host"] = host_product_baseline(seconds)
    return out


def host_product_baseline(seconds):
    """BASELINE C1 through THIS package on CPU tensors: MinMaxObserver.forward +
    UniformQuantizer.quantize take the native host loops (vsiquantization_amd/host.py,
    csrc/k_host.hip), the same op sequence the reference runs -- reported beside the
    reference's own timing, not used as the GPU's baseline."""
    import vsiquantization_amd as V
    from vsiquantization_amd import host
    x = torch.randn(256, 256, generator=torch.Generator().manual_seed(0))
    q = V.UniformQuantizer(8, True)

    def fn():
        s, z = V.MinMaxObserver(True).forward(x)
        return q.quantize(x, s, z, False)
    t, runs = _best_time(fn, seconds)
    return {"value": x.numel() / t / 1e6, "unit": "Melem/s", "us_per_call": 1e6 * t, "host_threads": host.threads(),
            "host_simd": host.simd(),
            "sample": f"the whole 256x256 C1 call (fresh observer, observe + fake quant), min of {runs} runs"}


# --------------------------------------------------------------------------- measurement
_T0 = time.perf_counter()


def progress(msg):
    """One line per phase on stderr (long runs must not look hung)."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def load_pmc_traffic(workload, kernel):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        return d[workload][kernel]["hbm_bytes_per_launch"]
    except Exception:  # noqa: BLE001
        return None


def settle_gates(W, cap=4000, world=1):
    """Untimed steps until the store-gate tuner (csrc/gate_tune.hip) has chosen the gate
    of every one-round launch site this workload uses: each site's first ~100 launches
    time candidate gates.  A choice of delay only -- results are identical for every gate.
    With several ranks the stop is agreed (MAX of the ranks' pending counts), so every
    rank runs the same steps -- a workload whose step holds a collective would otherwise
    hang.  The steps run in the timed region's pattern (launch_group: a group's forwards,
    then its backwards), so each site is tuned in the order its timed launches run in -- a
    K3 gate tuned between STE launches is up to 4 % slow for K3 launches that follow K3
    launches (tools/exp/c2_floor.py).  Returns (steps run, one dict per tuned site)."""
    from vsiquantization_amd import _hip as H
    grouped = hasattr(W, "launch_group")
    if grouped:
        g = max(1, int(W.group))
        ev = [timing_event() for _ in range(len(W.kernels) + 1)]
    n = 0
    while n < cap:   # at least one round, so that every launch site exists
        k = 0
        while k < 8:
            if grouped:
                assert W.launch_group(n, g, ev) == 0
                n, k = n + g, k + g
            else:
                assert W.launch(n) == 0
                n, k = n + 1, k + 1
        torch.cuda.synchronize()
        pending = H.gate_tuning_pending()
        if world > 1:
            on_gpu = dist.get_backend() == "nccl"
            p = torch.tensor([pending], dtype=torch.int64, device=torch.cuda.current_device() if on_gpu else "cpu")
            dist.all_reduce(p, op=dist.ReduceOp.MAX)
            pending = int(p)
        if pending == 0:
            break
    sites = []
    for line in H.gate_report().splitlines():
        f = line.split()
        kv = dict(x.split("=") for x in f[1:] if "=" in x)
        # every candidate gate the tuner timed at this site: [ticks, median us] (ticks 0 = no
        # gate), so a line shows whether another gate would have won on its box
        cands = [[int(t), float(us)] for t, us in (x.split(":") for x in f[1:] if ":" in x)]
        sites.append({"site": f[0], "grid": int(kv["grid"]), "read_bytes": int(kv["bytes"]),
                      "est_ticks": int(float(kv["est"])), "gate_ticks": int(kv["best"]),
                      "tuned": kv["done"] == "1", "retunes": int(kv.get("retunes", 0)), "candidates": cands})
    return n, sites


class _PhaseMark:
    """Stands in for the timing event k of a launch group while the group is captured:
    event 0 opens the first phase's HIP graph, event k closes phase k-1 and opens phase
    k, the last one closes the last phase (each phase of each group one graph)."""

    def __init__(self, cap, k, last):
        self.cap, self.k, self.last = cap, k, last

    def record(self, *_):
        cap = self.cap
        if self.k > 0:
            cap.ctx.__exit__(None, None, None)
            cap.graphs.append(cap.cur)
        if not self.last:
            cap.cur = torch.cuda.CUDAGraph()
            # thread_local: torch's NCCL watchdog thread keeps polling earlier collectives'
            # events during the capture (global mode makes that a capture error -> abort)
            cap.ctx = torch.cuda.graph(cap.cur, stream=cap.stream, capture_error_mode="thread_local")
            cap.ctx.__enter__()


class _GroupCapture:
    def __init__(self, stream):
        self.stream, self.graphs, self.cur, self.ctx = stream, [], None, None


def capture_groups(W, groups, nphase):
    """Every launch group of the timed region, phase by phase, as HIP graphs (the same
    launches, replayed without host work between the kernels).  None when a workload's
    launches cannot be captured (then the timed region launches directly)."""
    from vsiquantization_amd.utils.graph import quiesce_collectives
    stream = torch.cuda.current_stream()
    out = []
    # every collective captured below runs on its group's capture-only twin (RCCL), which
    # never runs an eager collective (vsiquantization_amd.distributed.prepare_capture)
    quiesce_collectives()
    try:
        for g0, cnt in groups:
            cap = _GroupCapture(stream)
            rc = W.launch_group(g0, cnt, [_PhaseMark(cap, k, k == nphase) for k in range(nphase + 1)])
            if rc != 0 or len(cap.graphs) != nphase:
                return None
            out.append(cap.graphs)
    except Exception as e:  # noqa: BLE001
        progress(f"graph capture not used: {type(e).__name__}: {e}")
        torch.cuda.synchronize()
        return None
    torch.cuda.synchronize()
    return out


def measure(W, steps, warmup, world, graphs=None):
    """W untimed warmup steps, self-check, then exactly `steps` timed steps between
    barrier + synchronize on both sides; the max over ranks of the wall time; per-phase
    HIP-event durations (rank-local) -> roofline of the dominant phase.

    Launch mode (one rank; graphs None = VSIQ_BENCH_GRAPH, default on): the timed launch
    groups are also captured as HIP graphs (after the warm-up and the store-gate settling,
    capture_groups).  Replaying them removes the host's per-launch cost (ctypes +
    hipLaunchKernel, 5-10 us on a slow host, comparable to a C2 kernel) from between the
    kernels, but a graph's kernel nodes dispatch a little slower than direct launches on a
    fast host (measured: C2 29.7 vs 28.2 us/step).  So an untimed trial (up to 4 groups,
    5 rounds each way, median wall time; one rank: graph unless direct is >1 % faster,
    several: graph only if >1 % faster) picks the mode for the timed region, and the same
    `steps` are then timed the other way too and reported as "alt_launch"."""
    for i in range(warmup):
        assert W.launch(i) == 0
    settle, gate_sites = settle_gates(W, world=world)
    names = list(W.kernels)
    ns = W.group
    groups = [(g0, min(ns, steps - g0)) for g0 in range(0, steps, ns)]
    if graphs is None:
        graphs = os.environ.get("VSIQ_BENCH_GRAPH", "1") == "1"
    # graphs under RCCL too: a step holding collectives (the act leg's per-layer all_gather,
    # C5's sync all-reduces) is captured whole, so the N > 1 timed region replays the
    # exchange with no host work between the kernels; gloo collectives are not capturable
    can = graphs and (world == 1 or dist.get_backend() == "nccl")
    captured = capture_groups(W, groups, len(names)) if can else None
    if world > 1 and not _agree(captured is not None, world):   # every rank captured, or none uses graphs
        captured = None
    use_graph, trial = False, None
    if captured is not None:
        use_graph, trial = _pick_launch(W, groups, captured, world=world)
        if world > 1:
            use_graph = _agree(use_graph, world)
    dt, evs = _timed(W, groups, names, steps, world, captured if use_graph else None)
    alt = _timed(W, groups, names, steps, world, None if use_graph else captured) if captured is not None else None
    out = _report(W, steps, world, dt, _durations(evs, names, steps), names, settle, gate_sites)
    out["launch"] = "hip graph per phase and group" if use_graph else "direct"
    if alt is not None:
        adt, aevs = alt
        ar = _report(W, steps, world, adt, _durations(aevs, names, steps), names, settle, gate_sites)
        out["alt_launch"] = {"launch": "direct" if use_graph else "hip graph per phase and group",
                             "value": ar["value"], "ms_per_step": ar["ms_per_step"],
                             "frac": ar["roofline"]["frac"],
                             "kernels_us": {k: v["avg_us"] for k, v in ar["kernels"].items()},
                             "trial_ms": trial}
    return out


def _agree(flag, world):
    """True only if `flag` is true on every rank (all-reduce MIN; RCCL tensors on the GPU,
    gloo on the CPU): ranks whose steps hold collectives must run the same launch mode."""
    if world <= 1:
        return bool(flag)
    on_gpu = dist.get_backend() == "nccl"
    t = torch.tensor([int(bool(flag))], dtype=torch.int64, device=torch.cuda.current_device() if on_gpu else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t))


def _durations(evs, names, steps):
    return {k: sum(e[i].elapsed_time(e[i + 1]) for e in evs) / steps * 1e-3 for i, k in enumerate(names)}


class _NoEvent:
    def record(self, *_):
        pass


def _pick_launch(W, groups, graphs, reps=5, margin=0.01, min_ms=20.0, max_reps=50, world=1):
    """Untimed trial: up to 4 launch groups each way, `reps` rounds -- more (up to
    `max_reps`) while the trial has run less than `min_ms` per mode, so that a short
    workload's (C1: ~0.25 ms per round) choice is not decided by host noise -- median
    wall time per mode; one rank: graph replay unless direct launches are faster by more
    than `margin`.  Several ranks: graph replay only when it is faster by more than
    `margin`, and exactly `reps` rounds (every rank runs the same collectives; the caller
    agrees on the choice).  Returns
    (use graph?, {mode: median ms})."""
    sel = list(range(min(4, len(groups))))
    t = {"direct": [], "graph": []}
    r = 0
    while r < reps or (world == 1 and r < max_reps and min(sum(t["direct"]), sum(t["graph"])) < min_ms):
        r += 1
        for mode in ("direct", "graph"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for j in sel:
                if mode == "graph":
                    for g in graphs[j]:
                        g.replay()
                else:
                    g0, cnt = groups[j]
                    assert W.launch_group(g0, cnt, [_NoEvent()] * (len(graphs[j]) + 1)) == 0
            torch.cuda.synchronize()
            t[mode].append((time.perf_counter() - t0) * 1e3)
    med = {k: sorted(v)[len(v) // 2] for k, v in t.items()}
    if world == 1:
        # one rank: graph replay unless direct launches are clearly faster -- within the
        # margin the replay wins, since it does not depend on the host keeping up (round 5:
        # C5 on a box whose host ran 2x slow: 417.9 us/step direct, 378.3 replayed, after a
        # trial that had them tied)
        return med["graph"] <= (1.0 + margin) * med["direct"], med
    return med["graph"] < (1.0 - margin) * med["direct"], med


class _Chained:
    """Timing event 0 of a launch group after the first: the previous group's last event,
    recorded right before this group's first launch -- consecutive groups share one
    marker on the stream instead of two (each marker is a packet between the kernels)."""

    def __init__(self, ev):
        self.ev = ev

    def record(self, *_):
        pass

    def elapsed_time(self, other):
        return self.ev.elapsed_time(other)


MARKERS = []   # [stream handle getter] when --markers: trace markers around each timed region


def _marker(end):
    if MARKERS:
        from vsiquantization_amd import _hip as H
        assert H.lib().vsiq_trace_marker(int(end), H.stream_of(torch.cuda.current_device())) == 0


def _timed(W, groups, names, steps, world, captured):
    chain = os.environ.get("VSIQ_BENCH_CHAIN", "1") == "1"
    evs = []
    for _ in groups:
        row = [timing_event() for _ in range(len(names) + 1)]
        if chain and evs:
            row[0] = _Chained(evs[-1][-1])
        evs.append(row)
    _marker(0)   # queued before the synchronize: outside the wall-clock window
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rc = 0
    if captured is None:
        for (g0, cnt), ev in zip(groups, evs):
            rc |= W.launch_group(g0, cnt, ev)
    else:
        for gr, ev in zip(captured, evs):
            ev[0].record()
            for k, g in enumerate(gr):
                g.replay()
                ev[k + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    _marker(1)
    assert rc == 0, f"kernel launch failed rc={rc}"
    return dt, evs


def _report(W, steps, world, dt, dur, names, settle, gate_sites):
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=torch.cuda.current_device())
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    # self-check AFTER the timed region, on the outputs of the timed launches (host work
    # between warmup and timing would leave the GPU idle right before the timed steps)
    ok = bool(W.check())
    if world > 1:
        t = torch.tensor([int(ok)], device=torch.cuda.current_device())
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        ok = bool(t.item())
    dom = max((k for k in names if W.kernels[k] > 0), key=dur.get)
    achieved = W.kernels[dom] / dur[dom] / 1e9
    per_kernel = {k: {"avg_us": dur[k] * 1e6, "alg_bytes": W.kernels[k],
                      "GBps": W.kernels[k] / dur[k] / 1e9 if dur[k] > 0 else 0.0,
                      "frac": W.kernels[k] / dur[k] / 1e9 / HBM_PEAK_GBS if dur[k] > 0 else 0.0}
                  for k in names}
    total = W.n * steps * world   # W.n: elements per rank per step (act: its 1/world of the batch)
    return {"value": total / dt / 1e6, "ms_per_step": dt / steps * 1e3, "self_check": ok,
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": load_pmc_traffic(W.key, dom),
                         # the whole timed step: every phase's algorithmic bytes over the
                         # wall time per step (launch gaps and host time included)
                         "step_frac": sum(W.kernels.values()) / (dt / steps) / 1e9 / HBM_PEAK_GBS},
            "kernels": per_kernel,
            "store_gate": {"settle_steps": settle, "sites": gate_sites}}


def gate_retunes(H):
    """Re-tunes of the store-gate sites so far (csrc/gate_tune.hip's drift monitor)."""
    return sum(int(t.split("=")[1]) for l in H.gate_report().splitlines() for t in l.split()
               if t.startswith("retunes="))


def _interleaved_us(fns, steps=100, reps=11, warmup=30):
    """Host + GPU time per call (us) of each step function, the reps interleaved so that
    both see the same host load: (median, min) per function."""
    for f in fns:
        for i in range(warmup):
            f(i)
    res = [[] for _ in fns]
    for r in range(reps):
        for k, f in enumerate(fns):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                f(i)
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) / steps * 1e6)
    return [(sorted(v)[len(v) // 2], min(v)) for v in res]


def api_timings(dev):
    """Public-API step timings, interleaved so every step function sees the same host load
    (host time on the shared boxes moves 2x between processes and minutes): median (and
    min) of 11 runs of 100 steps each, us per step.

    * api_us_per_step: the C2 step through the PUBLIC Python API (what a QAT user runs):
      PerChannelMinMaxObserver.observe_quantize(W, PerChannelUniformQuantizer(8, False)) +
      backward, fresh gradient per step, 4 weights in rotation (C++ autograd nodes,
      csrc/torch_ops.cpp);
    * api_torch_ref_us_per_step: torch's own trivial autograd step on the same tensors,
      (x * 1.0).backward(g) -- the floor of any public-API step on that box;
    * api_learn_us_per_step vs api_learn_torch_xs_us_per_step: the learnable per-call step,
      UniformQuantizer(4, True).quantize(x, s, 0, True) fwd + bwd (K1 + K4, f64 scale
      Parameter) against torch's own x * s fwd + bwd on one 8x16x20x20 activation."""
    import vsiquantization_amd as V
    gen = torch.Generator(device=dev).manual_seed(12)
    xs = [(torch.randn(C2PerChannel.shape, device=dev, generator=gen) * 0.05).requires_grad_(True)
          for _ in range(4)]
    g = torch.randn(C2PerChannel.shape, device=dev, generator=gen)
    obs, qpc = V.PerChannelMinMaxObserver(False), V.PerChannelUniformQuantizer(8, False)

    def ours(i):
        x = xs[i % 4]
        x.grad = None
        y, _ = obs.observe_quantize(x, qpc)
        y.backward(g)

    def trivial(i):
        x = xs[i % 4]
        x.grad = None
        (x * 1.0).backward(g)

    xa = torch.randn(8, 16, 20, 20, device=dev, generator=gen).requires_grad_(True)
    ga = torch.randn(8, 16, 20, 20, device=dev, generator=gen)
    q = V.UniformQuantizer(4, True)
    sc = torch.nn.Parameter(torch.tensor(0.05, dtype=torch.float64, device=dev))

    def learn(i):
        xa.grad = None
        sc.grad = None
        q.quantize(xa, sc, 0, True).backward(ga)

    def torch_xs(i):
        xa.grad = None
        sc.grad = None
        (xa * sc.float()).backward(ga)

    fns = [ours, trivial, learn, torch_xs]
    _interleaved_us(fns, reps=3)   # discarded: the first rounds after the GPU legs run on a cold host path
    (ou, ou_min), (tr, tr_min), (le, le_min), (tx, tx_min) = _interleaved_us(fns)
    return {"api_us_per_step": ou, "api_us_per_step_min": ou_min,
            "api_torch_ref_us_per_step": tr, "api_torch_ref_us_per_step_min": tr_min,
            "api_learn_us_per_step": le, "api_learn_us_per_step_min": le_min,
            "api_learn_torch_xs_us_per_step": tx, "api_learn_torch_xs_us_per_step_min": tx_min}


def api_graph_us_per_step(dev, steps=300):
    """The same public-API C2 step captured once with utils.graph.GraphedStep and replayed
    (the way to drop the per-step host cost of the Python API and torch's autograd engine):
    time per replay, median of 5 runs."""
    import vsiquantization_amd as V
    from vsiquantization_amd.utils.graph import GraphedStep
    shape = C2PerChannel.shape
    gen = torch.Generator(device=dev).manual_seed(11)
    w = (torch.randn(shape, device=dev, generator=gen) * 0.05).requires_grad_(True)
    g = torch.randn(shape, device=dev, generator=gen)
    obs, q = V.PerChannelMinMaxObserver(False), V.PerChannelUniformQuantizer(8, False)

    def step():
        y, _ = obs.observe_quantize(w, q)
        y.backward(g)
        return y

    gs = GraphedStep(step, grads_of=[w])
    reps = []
    for r in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps // 5):
            gs()
        torch.cuda.synchronize()
        reps.append((time.perf_counter() - t0) / (steps // 5) * 1e6)
    return sorted(reps)[2]


METRICS = {"c1": "Melements/s per-tensor observe + fake-quant fwd (256x256) + achieved HBM GB/s vs roofline",
           "c2": "Melements/s fake-quant fwd+bwd (per-channel int8) + achieved HBM GB/s vs roofline",
           "c3": "Melements/s LSQ fake-quant fwd+bwd + achieved HBM GB/s vs roofline",
           "c4": "Melements/s backbone fake-quant fwd+bwd (weights + fused ReLU/act) + achieved "
                 "HBM GB/s vs roofline",
           "c5": "Melements/s calibration pass (fused ReLU written + observer records, 27 layers, "
                 "deferred RCCL sync) + achieved HBM GB/s vs roofline",
           "act": "Melements/s batched activation observe + fake quant (per-call RCCL exchange) + "
                  "achieved HBM GB/s vs roofline"}


def build_workload(key, a, dev, rank, world):
    if key == "c4":
        return C4Backbone(dev, a.slots, 1000 * rank, batch=a.batch, bits_w=a.bits_w, bits_a=a.bits_a,
                          deferred=not a.per_call_grads)
    if key == "c5":
        return C5Calibration(dev, a.slots, 1000 * rank, batch=128, steps=16)
    if key == "act":
        return ActQuant(dev, world, rank)
    if key == "c3":
        return C3Lsq(dev, a.slots, 1000 * rank, asym=a.asym)
    return {"c1": C1PerTensor, "c2": C2PerChannel}[key](dev, a.slots, 1000 * rank)


def describe(W, key, a, world):
    cfg = {"workload": W.name, "shape": list(W.shape), "elements_per_step": W.n}
    if key in ("c1", "c2", "c3"):
        cfg.update(slots=len(W.slots), parallelism=f"replicas x{world} (independent tensors per rank, "
                                                   "no collective on this path)")
    if key == "c4":
        cfg.update(layers=len(W.layers), bits_w=W.bits[0], bits_a=W.bits[1],
                   act_elements_per_step=W.n_act, weight_elements_per_step=W.n_w,
                   act_scale_grads=("records-only K4 per layer + one fold launch (deferred)" if W.deferred
                                    else "folded inside each K4 launch"),
                   parallelism=f"dp x{world} (batch {a.batch} per GPU; quantizer path has no "
                               "collective, scale grads ride DDP's all-reduce)",
                   note="conv (MIOpen) excluded: synthetic conv outputs stand in for it")
    if key == "c5":
        cfg.update(layers=len(W.layers), images_per_gpu_per_batch=128, batches=16,
                   act_elements_per_batch=W.n,
                   parallelism=f"dp x{world} (128 images per GPU per batch; deferred observer sync: "
                               "2 all-reduces per calibration run)",
                   note="conv (MIOpen) excluded: synthetic conv outputs stand in for it")
    if key == "act":
        cfg.update(layers=len(W.layers), total_batch=ACT_BATCH, images_per_gpu=W.batch,
                   elements_per_gpu_per_step=W.n, bits_a=4, observer_bits=8,
                   parallelism=f"dp x{world} (batch {ACT_BATCH} split over the ranks; per layer one "
                               "RCCL all_gather of the observer stats records)" if world > 1 else "1 GPU, no exchange",
                   note="conv (MIOpen) excluded: synthetic conv outputs stand in for it")
    return cfg


def dry_run(a, world, rank):
    """Launcher rehearsal on the CPU: every rank joins a gloo group and contributes 1."""
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.ones(1)
        dist.all_reduce(t)
        ranks = int(t.item())
        dist.destroy_process_group()
    else:
        ranks = 1
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "requested_gpus": a.gpus, "ranks_joined": ranks}),
              flush=True)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        return launch_ranks(a, argv)
    world = int(env_world or 1)
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; launch with --nproc-per-node={a.gpus} "
              "or without torchrun", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.dry_run:
        dry_run(a, world, rank)
        return 0
    # VSIQ_BENCH_BACKEND=gloo + ranks sharing one GPU: rehearsal of the N>1 path on a
    # 1-GPU box only (the driver's multi-GPU runs use RCCL, one GPU per rank)
    backend = os.environ.get("VSIQ_BENCH_BACKEND", "nccl")
    dev = torch.device("cuda", local if backend == "nccl" else local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    # every launch of the run on one non-default stream (HIP graphs of the timed groups are
    # captured on it: measure / capture_groups)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()
        # the ranks that joined, counted by a real collective of this run (RCCL on the GPUs)
        t = torch.ones(1, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t)
        ranks_joined = int(t.item())
    else:
        ranks_joined = 1
    import vsiquantization_amd  # noqa: F401  (torch first, then the HIP library)
    from vsiquantization_amd import _hip as H
    for kv in a.tune:
        k, v = kv.split("=")
        H.set_tuning(int(k), int(v))
    if a.gate_table:
        progress(f"gate table {a.gate_table}: {H.gate_load(a.gate_table)} sites, tuner frozen")
    if a.markers:
        MARKERS.append(True)
    cpu = rank == 0 and world == 1 and not a.no_cpu_baseline
    bits = (a.bits_w, a.bits_a)

    progress(f"{a.workload}: build")
    W = build_workload(a.workload, a, dev, rank, world)
    progress(f"{a.workload}: measure")
    r = measure(W, a.steps, a.warmup, world)
    cfg = describe(W, a.workload, a, world)
    cfg["self_check"] = r["self_check"]
    out = {
        "metric": METRICS[a.workload],
        "value": r["value"],
        "unit": "Melem/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": r["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong" if a.workload == "act" else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (torch.randn, seeded per rank/slot)",
        "config": cfg,
        "roofline": r["roofline"],
        "kernels": r["kernels"],
        "store_gate": r["store_gate"],
        "launch": r["launch"],
        "timing_events": timing_events_kind(),
        "ranks_joined": ranks_joined,
        "backend": (dist.get_backend() if world > 1 else None),
    }
    if "alt_launch" in r:
        out["alt_launch"] = r["alt_launch"]
    if a.tune:
        out["config"]["tuning"] = a.tune
    if a.gate_table:
        out["store_gate"]["table"] = {"loaded": a.gate_table, "frozen": True}
    if a.workload == "c2":
        progress("c2: forward with uint8 codes")
        out["kernels"]["pc_observe_fq_fwd_with_codes"] = W.codes_variant()
    if hasattr(W, "alt_kernels"):
        out["kernels"].update(W.alt_kernels())
    del W
    torch.cuda.empty_cache()
    if a.workload == "c2" and not a.no_api:
        progress("c2: public API timing")
        r0 = gate_retunes(H)
        out.update(api_timings(dev))
        out["api_gate_retunes"] = gate_retunes(H) - r0
        out["api_graph_us_per_step"] = api_graph_us_per_step(dev)
        torch.cuda.empty_cache()

    extras = {}
    for key in a.extras:
        if key == a.workload:
            continue
        steps, warm = EXTRA_STEPS[key]
        progress(f"{key}: build + measure")
        try:
            Wx = build_workload(key, a, dev, rank, world)
            rx = measure(Wx, steps, warm, world)
            if hasattr(Wx, "alt_kernels"):
                rx["kernels"].update(Wx.alt_kernels())
        except Exception as e:  # noqa: BLE001
            # a secondary leg that fails (on every rank alike) must not cost the
            # headline line: record the error in its place and go on
            progress(f"{key}: FAILED {e!r}"[:400])
            extras[key] = {"metric": METRICS[key], "error": repr(e)[:400]}
            Wx = None
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            continue
        extras[key] = {"metric": METRICS[key], "value": rx["value"], "unit": "Melem/s",
                       "ms_per_step": rx["ms_per_step"], "steps": steps, "warmup": warm,
                       "scaling": "strong" if key == "act" else "weak",
                       "config": dict(describe(Wx, key, a, world), self_check=rx["self_check"]),
                       "roofline": rx["roofline"], "kernels": rx["kernels"], "launch": rx["launch"]}
        if "alt_launch" in rx:
            extras[key]["alt_launch"] = rx["alt_launch"]
        del Wx
        torch.cuda.empty_cache()
    if a.save_gate_table and rank == 0:
        progress(f"gate table saved: {H.gate_save(a.save_gate_table)} sites -> {a.save_gate_table}")
    if cpu:
        # CPU legs after every GPU measurement (host threads do not disturb the timed regions)
        cpu_key = lambda k: "c3asym" if k == "c3" and a.asym else k   # noqa: E731
        out["cpu_baseline"] = cpu_baseline(cpu_key(a.workload), a.cpu_seconds, bits)
        for key, e in extras.items():
            if "error" not in e:
                e["cpu_baseline"] = cpu_baseline(cpu_key(key), a.cpu_seconds, bits)
    if "act" in extras:
        out["batched_act_quant"] = extras.pop("act")
    if extras:
        out["configs"] = extras
    if rank == 0:
        print(json.dumps(out), flush=True)
        print(compact_summary(out), file=sys.stderr, flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def compact_summary(out) -> str:
    """The line's key figures in a few hundred characters on stderr (after the JSON line):
    a driver that keeps only the tail of a long line still records every config's value
    and roofline fraction, the public-API timings and the chosen store gates."""
    def leg(name, d):
        if "error" in d:
            return f"{name} FAILED {d['error'][:120]}"
        ks = ",".join(f"{k}={v['frac']:.3f}" + ("" if v.get("in_step", True) else "*")
                      for k, v in d.get("kernels", {}).items() if isinstance(v, dict) and v.get("frac"))
        cb = (d.get("cpu_baseline") or {}).get("value")
        sf = (d.get("roofline") or {}).get("step_frac")
        return (f"{name} {d['value']:.1f}Melem/s {1e3 * d['ms_per_step']:.2f}us {d.get('launch', '')[:6]} [{ks}]"
                + (f" step={sf:.3f}" if sf else "") + (f" cpu={cb:.1f}" if cb else ""))
    parts = [leg(out["config"].get("workload", "")[:2], out)]
    parts += [leg(k, v) for k, v in (out.get("configs") or {}).items()]
    if "batched_act_quant" in out:
        parts.append(leg("act", out["batched_act_quant"]))
    api = {k: round(v, 1) for k, v in out.items() if k.startswith("api_") and isinstance(v, (int, float))}
    def gate(s):   # chosen gate (its median us / the no-gate median us)
        c = dict((t, us) for t, us in s.get("candidates", []))
        if s["gate_ticks"] in c and 0 in c:
            return f"{s['site']}:{s['gate_ticks']}({c[s['gate_ticks']]:.2f}/{c[0]:.2f}us)"
        return f"{s['site']}:{s['gate_ticks']}"
    gates = ",".join(gate(s) for s in out.get("store_gate", {}).get("sites", []))
    return "[bench summary] " + " | ".join(parts) + f" | api {api} | gates {gates}"


if __name__ == "__main__":
    sys.exit(main())
