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
    p.add_argument("--workload", choices=["c1", "c2", "c3", "c4", "c5"], default="c2")
    p.add_argument("--batch", type=int, default=256, help="C4 batch (reference: 256)")
    p.add_argument("--bits-w", type=int, default=2, help="C4 weight bits (YAML default 2; SURVEY also w8)")
    p.add_argument("--bits-a", type=int, default=4, help="C4 activation bits (YAML default 4; SURVEY also a8)")
    p.add_argument("--slots", type=int, default=8)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                   help="experiments: vsiq_set_tuning(KEY, VALUE) before the workload is built "
                        "(keys: include/vsiq.h VSIQ_TUNE_*)")
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


class C1PerTensor:
    """C1: the reference's minimal config -- MinMaxObserver + UniformQuantizer, per-tensor
    symmetric int8, on a 256x256 fp32 weight (observers/minmax.py:76-88 then
    quantizers/uniform.py:34-56): per step one K2 observe (running min/max + f64 qparams
    on the device) and one K1 fake quant reading those qparams by pointer.  65,536
    elements: latency-bound (launch + reduction chain), the GB/s are not the point."""

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
        self.f_fwd = lib.vsiq_observe_f32
        self.f_bwd = lib.vsiq_fq_fwd_f32
        self.kernels = {"observe": 4 * n, "fq_fwd": 8 * n}

    launch = None   # set below (same group structure as C2: all observes, then all fake quants)

    def check(self):
        """Slot 0 against the reference's formulas in torch on the host (IEEE fp32 x / s)."""
        s = self.slots[0]
        x = s["x"].cpu()
        mn, mx = min(0.0, float(x.min())), max(0.0, float(x.max()))
        scale = max(abs(mn), abs(mx)) / (2 ** 7 - 1 + 1e-8)
        want = torch.clamp(torch.round(x / scale), -128, 127) * scale
        return bool(torch.equal(s["y"].cpu().view(torch.int32), want.view(torch.int32)))


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


C1PerTensor.launch = C2PerChannel.launch
C1PerTensor.launch_group = C2PerChannel.launch_group


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


class C4Backbone:
    """C4: the YOLOv8n backbone's 27 ConvBnReLU quantizers at 320x320, batch 256, in the
    learning phase: the 27 learnable weight fake quants as one multi-tensor launch each way
    (k_multi.hip, the path of enable_multi_tensor_weights) and per layer the fused ReLU +
    learnable activation fake quant (K5: K1-relu fwd, K4-relu bwd).  The conv itself is
    MIOpen and out of scope: synthetic conv outputs of the right shapes stand in for it."""

    name = "C4 YOLOv8n backbone ConvBnReLU fake-quant (weights + fused ReLU/act), learnable"

    def __init__(self, dev, slots, seed_base, batch=256, bits_w=2, bits_a=4):
        from vsiquantization_amd import _hip as H
        self.H = H
        lib = H.lib()
        st = H.stream_of(dev)
        self.layers = yolov8n_backbone()
        self.shape = (batch, 3, 320, 320)
        qw = (-(2 ** (bits_w - 1)), 2 ** (bits_w - 1) - 1)
        qa = (-(2 ** (bits_a - 1)), 2 ** (bits_a - 1) - 1)
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
        """grad scale of the first activation quantizer is finite and the fused ReLU zeroed
        the gradient wherever the conv output is negative."""
        t = self.keep[0]
        neg = t["c"] < 0
        return bool(torch.isfinite(t["grads_a"]).all()) and bool((t["gc"][neg] == 0).all())


class C5Calibration:
    """C5: calibration of the YOLOv8n backbone's 27 activation quantizers (MinMaxObserver,
    sym) on batches of 128 images per GPU (1024 over 8 GPUs): per batch and layer one
    deferred observer pass over the fused ReLU of the conv output (K2p-relu, 4 B/elem
    read), each writing its partial records into its own device slot (no fold, no
    atomics, no sync); after the last batch ONE deferred sync -- one fold launch over all
    slots of all layers and batches, two RCCL all-reduces over the records, and the exact
    replay of every layer's running min/max (the path of calibrate_qat_model(...,
    defer_observers=True) / QuantizationManager.dist_defer + distributed.sync_calibration,
    here driven through the C ABI so the Python manager's per-call host cost is not what
    is measured).  min/max are bit-identical to a 1-GPU run (tests/test_dist_gloo.py).
    Synthetic conv outputs stand in for the conv (MIOpen, out of scope)."""

    name = "C5 YOLOv8n backbone calibration: fused-ReLU MinMax observers, deferred RCCL sync"

    def __init__(self, dev, slots, seed_base, batch=128, steps=16):
        from vsiquantization_amd import _hip as H
        from vsiquantization_amd.fakequant import qden
        self.H = H
        lib = H.lib()
        self.st = H.stream_of(dev)
        self.layers = yolov8n_backbone()
        self.shape = (batch, 3, 320, 320)
        gen = torch.Generator(device=dev).manual_seed(seed_base)
        self.acts = [torch.randn(batch, co, h, h, device=dev, generator=gen) for _, co, _, _, h in self.layers]
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.steps = steps
        L = len(self.layers)
        from vsiquantization_amd.fakequant import part_slot_doubles
        self.stride = max(part_slot_doubles(a.numel()) for a in self.acts)
        self.parts = torch.zeros(steps, L, self.stride, dtype=torch.float64, device=dev)
        self.f = lib.vsiq_act_observe_part_f32
        self.ptrs = [H.ptr(a) for a in self.acts]
        self.n = sum(a.numel() for a in self.acts)
        self.slots = [None]
        self.kernels = {"observe_all_layers": 4 * self.n, "sync": 0}
        self.minmax = None

    def _observe(self, step):
        H = self.H
        rc = 0
        base = self.parts[step % self.steps]
        for j, (p, a) in enumerate(zip(self.ptrs, self.acts)):
            rc |= self.f(p, H.c_i64(a.numel()), H.ACT_RELU, H.ptr(base[j]), H.c_i64(self.stride), self.st)
        return rc

    def launch(self, i):
        return self._observe(i)

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

    def launch_group(self, i0, cnt, ev):
        rc = 0
        ev[0].record()
        for j in range(cnt):
            rc |= self._observe(i0 + j)
        ev[1].record()
        self._sync(min(self.steps, i0 + cnt))
        ev[2].record()
        return rc

    def check(self):
        """Running min/max after the sync identical on every rank; equal to a direct
        reduction of the (synthetic) relu(conv output) on one GPU."""
        self._sync(1)
        mm = torch.stack(self.minmax, dim=-1)
        if self.world > 1:
            hi, lo = mm.clone(), mm.clone()
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            return bool(torch.equal(hi, lo))
        ref = [(min(0.0, float(torch.relu(a).min())), max(0.0, float(torch.relu(a).max()))) for a in self.acts]
        return [tuple(r) for r in mm.tolist()] == ref


# --------------------------------------------------------------------------- CPU baseline
def cpu_baseline(workload, seconds, bits=(2, 4)):
    """The reference's eager-torch op sequence (oracle/eager_torch.py) on the host cores."""
    from oracle import eager_torch as E
    threads = max(1, min(16, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    gen = torch.Generator().manual_seed(0)
    if workload == "c1":
        from oracle.fakequant_np import minmax_qparams
        x = torch.randn(256, 256, generator=gen)

        def fn():   # observers/minmax.py:76-88 (two .item()) then uniform.py:54-55,95
            mn, mx = E.observe(x)
            s, z = minmax_qparams(mn, mx, True, 8)
            return E.fake_quant(x, s, z, -128, 127)
        n = x.numel()
        sample = "the whole 256x256 workload (observe + fake quant per call)"
    elif workload == "c2":
        rows = 64   # bounded sample: 64 of the 1024 out-channels (same row length 9216)
        w = torch.randn(rows, 1024, 3, 3, generator=gen) * 0.05
        g = torch.randn(rows, 1024, 3, 3, generator=gen)
        fn = lambda: E.per_channel_step(w, g, symmetric=False, bits=8)  # noqa: E731
        n = w.numel()
        sample = f"{rows} of 1024 out-channels of the 1024x1024x3x3 weight (9216 elem/row), fwd+bwd"
    elif workload == "c5":
        imgs = 4   # bounded sample: 4 of the 128 images per GPU, all 27 layers

        acts = [torch.randn(imgs, co, h, h, generator=gen) for _, co, _, _, h in yolov8n_backbone()]

        def fn():   # reference calibration per layer: relu, observer (2 .item()), 3 stats
            for c in acts:
                a = torch.relu(c)
                E.observe(a)
                a.abs().mean().item(), a.mean().item(), a.std().item()
        n = sum(t.numel() for t in acts)
        sample = f"{imgs} of 128 images per GPU through all 27 backbone observers (relu + MinMax + stats)"
    elif workload == "c4":
        imgs = 4   # bounded sample: 4 of the 256 images, all 27 layers + their weights
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
        n = sum(t[0].numel() + t[2].numel() for t in tens)
        sample = f"{imgs} of 256 images through all 27 backbone layers (+ weights), w{bits[0]}/a{bits[1]}, fwd+bwd"
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
    # VSIQ_BENCH_BACKEND=gloo + ranks sharing one GPU: rehearsal of the N>1 path on a
    # 1-GPU box only (the driver's multi-GPU runs use RCCL, one GPU per rank)
    backend = os.environ.get("VSIQ_BENCH_BACKEND", "nccl")
    dev = torch.device("cuda", local if backend == "nccl" else local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    import vsiquantization_amd  # noqa: F401  (torch first, then the HIP library)
    from vsiquantization_amd import _hip as H
    for kv in a.tune:
        k, v = kv.split("=")
        H.set_tuning(int(k), int(v))

    if a.workload == "c4":
        W = C4Backbone(dev, a.slots, 1000 * rank, batch=a.batch, bits_w=a.bits_w, bits_a=a.bits_a)
    elif a.workload == "c5":
        W = C5Calibration(dev, a.slots, 1000 * rank, batch=128, steps=max(a.steps, a.warmup))
    else:
        W = {"c1": C1PerTensor, "c2": C2PerChannel, "c3": C3Lsq}[a.workload](dev, a.slots, 1000 * rank)
    for i in range(a.warmup):
        assert W.launch(i) == 0
    torch.cuda.synchronize()
    ok = W.check()

    ns = len(W.slots) if a.workload not in ("c4", "c5") else (4 if a.workload == "c4" else 16)
    # C4: events around 4 steps' phases; C5: 16 calibration batches, then the deferred sync
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
                      "GBps": W.kernels[k] / dur[k] / 1e9 if dur[k] > 0 else 0.0,
                      "frac": W.kernels[k] / dur[k] / 1e9 / HBM_PEAK_GBS if dur[k] > 0 else 0.0}
                  for k in names}

    total_elems = W.n * a.steps * world
    metrics = {"c1": "Melements/s per-tensor observe + fake-quant fwd (256x256) + achieved HBM GB/s vs roofline",
               "c2": "Melements/s fake-quant fwd+bwd (per-channel int8) + achieved HBM GB/s vs roofline",
               "c3": "Melements/s LSQ fake-quant fwd+bwd + achieved HBM GB/s vs roofline",
               "c4": "Melements/s backbone fake-quant fwd+bwd (weights + fused ReLU/act) + achieved "
                     "HBM GB/s vs roofline",
               "c5": "Melements/s calibration observer pass (fused ReLU, 27 layers, deferred RCCL "
                     "sync) + achieved HBM GB/s vs roofline"}
    out = {
        "metric": metrics[a.workload],
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
    if a.workload == "c4":
        out["config"].update(layers=len(W.layers), bits_w=W.bits[0], bits_a=W.bits[1],
                             act_elements_per_step=W.n_act, weight_elements_per_step=W.n_w,
                             parallelism=f"dp x{world} (batch {a.batch} per GPU; quantizer path has no "
                                         "collective, scale grads ride DDP's all-reduce)",
                             note="conv (MIOpen) excluded: synthetic conv outputs stand in for it")
    if a.workload == "c5":
        out["config"].update(layers=len(W.layers), images_per_gpu_per_batch=128,
                             batches=a.steps, act_elements_per_batch=W.n,
                             parallelism=f"dp x{world} (128 images per GPU per batch; deferred "
                                         "observer sync: 2 all-reduces per calibration run)",
                             note="conv (MIOpen) excluded: synthetic conv outputs stand in for it")
    if a.tune:
        out["config"]["tuning"] = a.tune
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.workload, a.cpu_seconds, bits=(a.bits_w, a.bits_a))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
