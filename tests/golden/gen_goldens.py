#!/usr/bin/env python3
"""Generate golden input/output vectors by running the REFERENCE's own CPU path.

This script is the only place that imports the reference implementation
(`/root/reference`, tranngocduvnvp/VSIQuantization @ 2025-08-08, PyTorch
2.10.0+rocm7.0 on CPU).  It runs in the build container only; the fixtures it
writes (`tests/golden/*.npz` + `cases.json`) are plain numeric data and travel
to the GPU box, the reference does not.

Reference call sites exercised (file:line under /root/reference):
  * observers/minmax.py:32-88          MinMaxObserver.observe / get_scale_zero_point / forward
  * quantizers/uniform.py:34-56        UniformQuantizer.quantize (fixed + learnable)
  * quantizers/uniform.py:81-96        discreate_tensor (the integer codes)
  * quantizers/uniform.py:242-271      ScaleGradient / RoundStraightThrough (autograd)
  * quantizers/quantization_manager.py:55-114  collect / quantize / learn-init sequence
  * modules/fused.py:32-134 + modules/fuse.py:45-149  (toy fused model, host structure)
  * modules/fused.py:133 + quantizers/fake_quantize.py:49-50  (F.relu / F.silu, then quantize_out)
  * modules/fused.py:32-412 (BN fold, fused forward/backward) + modules/fuse.py:45-149 /
    fuse_config.py:57-149 (fuse_modules_unified structure, child-name config lookup)

Per-channel has no reference class: it is defined as the
reference classes applied independently to each out-channel slice W[c].

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_goldens.py
"""
import json
import os
import sys
import types

sys.dont_write_bytecode = True
REF = os.environ.get("VSIQ_REFERENCE", "/root/reference")
sys.path.insert(0, REF)
# modules/fused.py:2-3 has dead imports of tkinter/turtle (absent here).
for _m, _attr in (("tkinter", "W"), ("turtle", "forward")):
    if _m not in sys.modules:
        _mod = types.ModuleType(_m)
        setattr(_mod, _attr, None)
        sys.modules[_m] = _mod

import numpy as np  # noqa: E402
import torch  # noqa: E402

from observers.minmax import MinMaxObserver  # noqa: E402
from quantizers.uniform import UniformQuantizer  # noqa: E402
from quantizers.quantization_manager import QuantizationManager  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
arrays = {}
cases = []


def put(key, t):
    a = t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)
    arrays[key] = np.ascontiguousarray(a)
    return key


def special_vector(n_rand, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n_rand, generator=g) * scale


# ---------------------------------------------------------------------------
# 1. Per-tensor observe + fake-quant (the §3.4 "observer + quantize" pair)
#    MinMaxObserver(sym, num_bits=obs_bits).forward(x) -> (s, zp);
#    UniformQuantizer(bits, sym).quantize(x, s, zp, False); backward with g.
# ---------------------------------------------------------------------------
def per_tensor_inputs():
    ins = {}
    g = torch.Generator().manual_seed(0)
    ins["randn"] = torch.randn(2, 3, 5, 7, generator=g)
    ins["pos"] = torch.rand(4, 33, generator=g) * 3.0 + 0.5
    ins["neg"] = -(torch.rand(4, 33, generator=g) * 2.0 + 0.25)
    ins["zeros"] = torch.zeros(3, 17)
    t = torch.randn(257, generator=g)
    t[5] = float("nan")
    ins["nan"] = t
    t = torch.randn(130, generator=g)
    t[7] = float("inf")
    ins["posinf"] = t
    t = torch.randn(130, generator=g)
    t[9] = float("-inf")
    ins["neginf"] = t
    t = torch.randn(1000, generator=g) * 0.05
    t[0] = -0.0
    t[1] = 0.0
    t[2] = 1e-40   # denormal
    t[3] = -1e-40
    ins["mixed"] = t
    return ins


def run_observe_fq(x, sym, bits, obs_bits):
    obs = MinMaxObserver(sym, obs_bits)
    rec = {}
    try:
        s, zp = obs.forward(x)
    except Exception as e:  # reference raises on non-finite zp (python round)
        rec["raises"] = type(e).__name__
        rec["min_val"] = float(obs.min_val)
        rec["max_val"] = float(obs.max_val)
        return rec, None
    rec.update(min_val=float(obs.min_val), max_val=float(obs.max_val),
               scale=float(s), zp=int(zp))
    q = UniformQuantizer(bits, sym)
    xr = x.clone().requires_grad_(True)
    y = q.quantize(xr, s, zp, False)
    x_int = q.discreate_tensor(x, s, zp, q.qmin, q.qmax)
    gg = torch.randn(x.shape, generator=torch.Generator().manual_seed(1234))
    y.backward(gg)
    return rec, (y.detach(), x_int, gg, xr.grad.detach())


idx = 0
for name, x in per_tensor_inputs().items():
    for sym in (True, False):
        for bits in (2, 4, 8):
            for obs_bits in ({8, bits} if bits != 8 else {8}):
                rec, outs = run_observe_fq(x, sym, bits, obs_bits)
                key = f"pt{idx}"
                idx += 1
                rec.update(kind="per_tensor_observe_fq", key=key, input=name,
                           sym=sym, bits=bits, obs_bits=obs_bits,
                           x=put(key + "_x", x))
                if outs is not None:
                    y, x_int, gg, gx = outs
                    rec.update(y=put(key + "_y", y), x_int=put(key + "_xint", x_int),
                               g=put(key + "_g", gg), grad_x=put(key + "_gx", gx))
                cases.append(rec)

# ---------------------------------------------------------------------------
# 2. Fixed-qparam fake-quant with hand-picked scale/zp (ties, clamp edges).
# ---------------------------------------------------------------------------
fixed_idx = 0
for sym in (True, False):
    for bits in (2, 4, 8):
        q = UniformQuantizer(bits, sym)
        for s in (0.25, 0.1, 1.0e-3, 3.0517578125e-05):
            for zp in ((0, 1) if sym else (0, 3, (q.qmax + 1) // 2)):
                ks = torch.arange(q.qmin - 3, q.qmax + 4, dtype=torch.float64)
                # exact ties (k+0.5)*s, integers and neighbours, in units of s
                grid = torch.cat([ks, ks + 0.5, ks - 0.5, ks + 0.49999, ks + 0.50001])
                x = ((grid - zp) * s).float()
                g = torch.Generator().manual_seed(99)
                x = torch.cat([x, torch.randn(200, generator=g) * s * (q.qmax - q.qmin) / 3,
                               torch.tensor([float("nan"), float("inf"), -float("inf"), 0.0, -0.0])])
                xr = x.clone().requires_grad_(True)
                y = q.quantize(xr, s, zp, False)
                x_int = q.discreate_tensor(x, s, zp, q.qmin, q.qmax)
                gg = torch.randn(x.shape, generator=torch.Generator().manual_seed(7))
                y.backward(gg)
                key = f"fx{fixed_idx}"
                fixed_idx += 1
                cases.append(dict(kind="fixed_fq", key=key, sym=sym, bits=bits, scale=s, zp=zp,
                                  x=put(key + "_x", x), y=put(key + "_y", y),
                                  x_int=put(key + "_xint", x_int), g=put(key + "_g", gg),
                                  grad_x=put(key + "_gx", xr.grad)))

# ---------------------------------------------------------------------------
# 3. Per-channel (axis 0 of OIHW): reference classes looped over out-channels.
# ---------------------------------------------------------------------------
def per_channel_weight(seed, special):
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(8, 4, 3, 3, generator=g) * 0.05
    if special:
        w[1] = w[1].abs() + 0.01         # all positive
        w[2] = -(w[2].abs() + 0.01)      # all negative
        w[3] = 0.0                        # all zero -> scale 0
        w[4, 0, 1, 1] = float("nan")     # NaN row: observer skips the call
        w[5, 1, 0, 2] = float("inf")     # +inf
    return w


pc_idx = 0
for special in (False, True):
    for sym in (True, False):
        for bits in (2, 4, 8):
            w = per_channel_weight(11 + pc_idx, special)
            if special and sym:
                w[6, 2, 2, 2] = -float("inf")  # -inf only for sym (asym raises in round())
            q = UniformQuantizer(bits, sym)
            gg = torch.randn(w.shape, generator=torch.Generator().manual_seed(5))
            ys, xis, gxs, scales, zps, mins, maxs = [], [], [], [], [], [], []
            for c in range(w.shape[0]):
                obs = MinMaxObserver(sym)  # fresh observer per channel per call, num_bits=8
                s, zp = obs.forward(w[c])
                xr = w[c].clone().requires_grad_(True)
                y = q.quantize(xr, s, zp, False)
                y.backward(gg[c])
                ys.append(y.detach())
                xis.append(q.discreate_tensor(w[c], s, zp, q.qmin, q.qmax))
                gxs.append(xr.grad.detach())
                scales.append(float(s))
                zps.append(int(zp))
                mins.append(float(obs.min_val))
                maxs.append(float(obs.max_val))
            key = f"pc{pc_idx}"
            pc_idx += 1
            cases.append(dict(kind="per_channel_observe_fq", key=key, sym=sym, bits=bits, obs_bits=8,
                              special=special, x=put(key + "_x", w), y=put(key + "_y", torch.stack(ys)),
                              x_int=put(key + "_xint", torch.stack(xis)), g=put(key + "_g", gg),
                              grad_x=put(key + "_gx", torch.stack(gxs)),
                              scale=put(key + "_scale", torch.tensor(scales, dtype=torch.float64)),
                              zp=put(key + "_zp", torch.tensor(zps, dtype=torch.int64)),
                              min_val=put(key + "_min", torch.tensor(mins, dtype=torch.float64)),
                              max_val=put(key + "_max", torch.tensor(maxs, dtype=torch.float64))))

# ---------------------------------------------------------------------------
# 4. Learnable (LSQ) path: quantize(x, Parameter f64 scale, zp, True) fwd + bwd.
# ---------------------------------------------------------------------------
lsq_idx = 0
for shape, seed in (((3, 4, 8, 8), 21), ((16, 3, 16, 16), 22)):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(shape, generator=g)
    gg = torch.randn(shape, generator=torch.Generator().manual_seed(seed + 100))
    for sym in (True, False):
        for bits in ((2, 4, 8) if x.numel() < 5000 else (8,)):
            q = UniformQuantizer(bits, sym)
            scale = torch.nn.Parameter(torch.tensor(np.float64(0.03 if bits == 8 else 0.3)))
            xr = x.clone().requires_grad_(True)
            if sym:
                zp = 0
                y = q.quantize(xr, scale, zp, True)
            else:
                zp = torch.nn.Parameter(torch.tensor(np.float64(3.0 if bits > 2 else 1.0) + 1e-9))
                y = q.quantize(xr, scale, zp, True)
            y.backward(gg)
            key = f"lsq{lsq_idx}"
            lsq_idx += 1
            rec = dict(kind="learnable_fq", key=key, sym=sym, bits=bits,
                       scale=float(scale.detach()), scale_grad=float(scale.grad),
                       x=put(key + "_x", x), g=put(key + "_g", gg),
                       y=put(key + "_y", y), grad_x=put(key + "_gx", xr.grad))
            if not sym:
                rec.update(zp=float(zp.detach()), zp_grad=float(zp.grad))
            else:
                rec.update(zp=0)
            cases.append(rec)

# 4b. calib_grad_scale as a per-channel fp32 tensor (utils/estimate_bn.py:136 sets it on the
#     activation quantizer): ScaleGradient's tensor-valued gradient (uniform.py:47-53,252-253)
#     is sum-reduced onto the 0-dim scale / zero point by autograd.
calib_idx = 0
for sym, bits in ((True, 8), (False, 8), (True, 4)):
    g = torch.Generator().manual_seed(40 + calib_idx)
    x = torch.randn((6, 5, 7, 7), generator=g)
    gg = torch.randn((6, 5, 7, 7), generator=g)
    calib = torch.rand(5, generator=g) * 2 + 0.1
    q = UniformQuantizer(bits, sym)
    q.calib_grad_scale = calib
    scale = torch.nn.Parameter(torch.tensor(np.float64(0.04 if bits == 8 else 0.3)))
    zp = 0 if sym else torch.nn.Parameter(torch.tensor(np.float64(5.0)))
    xr = x.clone().requires_grad_(True)
    y = q.quantize(xr, scale, zp, True)
    y.backward(gg)
    key = f"lsqc{calib_idx}"
    calib_idx += 1
    rec = dict(kind="learnable_fq_calib", key=key, sym=sym, bits=bits, scale=float(scale.detach()),
               scale_grad=float(scale.grad), calib=put(key + "_calib", calib),
               x=put(key + "_x", x), g=put(key + "_g", gg), y=put(key + "_y", y),
               grad_x=put(key + "_gx", xr.grad))
    if not sym:
        rec.update(zp=float(zp.detach()), zp_grad=float(zp.grad))
    else:
        rec.update(zp=0)
    cases.append(rec)

# 4c. symmetric quantizer + learnable scale + a gradient-requiring TENSOR zero point: the
#     symmetric branch skips zero_point_rounding / ScaleGradient (uniform.py:50-52), but
#     autograd still reaches zp through x/scale + zero_point and (x_int - zero_point) * scale
#     (uniform.py:54-55, 95): zp used as given, integer or not, inside or outside [qmin, qmax].
symzp_idx = 0
for bits, zpv in ((8, 0.0), (8, 3.0), (8, 1.3), (4, -2.0), (4, 0.75), (4, 9.0), (2, 0.0)):
    g = torch.Generator().manual_seed(60 + symzp_idx)
    x = torch.randn((4, 3, 9, 9), generator=g)
    gg = torch.randn((4, 3, 9, 9), generator=g)
    q = UniformQuantizer(bits, True)
    scale = torch.nn.Parameter(torch.tensor(np.float64(0.03 if bits == 8 else 0.3)))
    zp = torch.nn.Parameter(torch.tensor(np.float64(zpv)))
    xr = x.clone().requires_grad_(True)
    y = q.quantize(xr, scale, zp, True)
    y.backward(gg)
    key = f"lsqz{symzp_idx}"
    symzp_idx += 1
    cases.append(dict(kind="learnable_fq_sym_tensor_zp", key=key, sym=True, bits=bits,
                      scale=float(scale.detach()), scale_grad=float(scale.grad), zp=zpv,
                      zp_grad=float(zp.grad), x=put(key + "_x", x), g=put(key + "_g", gg),
                      y=put(key + "_y", y), grad_x=put(key + "_gx", xr.grad)))

# 4d. Learnable per-channel (axis 0), by SURVEY §0.2's definition: the reference's
#     learnable UniformQuantizer.quantize applied to each out-channel row W[c] with its own
#     0-dim f64 scale Parameter (and, asymmetric, its own f64 zero-point Parameter, which
#     zero_point_rounding rounds / clamps); ScaleGradient's factor is then the row's
#     (qmax * numel(W[c])) ** -0.5 (uniform.py:58-71).
pcl_idx = 0
for sym, bits in ((True, 8), (True, 4), (False, 8), (False, 4)):
    g = torch.Generator().manual_seed(80 + pcl_idx)
    w = torch.randn(6, 5, 3, 3, generator=g) * 0.2
    w[1] *= 8.0                                   # a row that clamps
    gg = torch.randn(w.shape, generator=g)
    q = UniformQuantizer(bits, sym)
    s0 = (torch.rand(6, generator=g) * 0.02 + 0.01).double() * (1.0 if bits == 8 else 8.0)
    z0 = [0.0] * 6 if sym else [3.0, 7.0, 0.0, 12.0, 1.0, 200.0]
    ys, gxs, gss, gzs = [], [], [], []
    for c in range(w.shape[0]):
        sc = torch.nn.Parameter(s0[c].clone())
        zc = 0 if sym else torch.nn.Parameter(torch.tensor(np.float64(z0[c])))
        xr = w[c].clone().requires_grad_(True)
        y = q.quantize(xr, sc, zc, True)
        y.backward(gg[c])
        ys.append(y.detach())
        gxs.append(xr.grad.detach())
        gss.append(float(sc.grad))
        gzs.append(0.0 if sym else float(zc.grad))
    key = f"pcl{pcl_idx}"
    pcl_idx += 1
    cases.append(dict(kind="per_channel_learnable", key=key, sym=sym, bits=bits, x=put(key + "_x", w),
                      g=put(key + "_g", gg), scale=put(key + "_scale", s0),
                      zp=put(key + "_zp", torch.tensor(z0, dtype=torch.float64)),
                      y=put(key + "_y", torch.stack(ys)), grad_x=put(key + "_gx", torch.stack(gxs)),
                      scale_grad=put(key + "_gs", torch.tensor(gss, dtype=torch.float64)),
                      zp_grad=put(key + "_gz", torch.tensor(gzs, dtype=torch.float64))))

# asym + learnable through the manager crashes in the reference (int zp -> torch.round(int)):
try:
    q = UniformQuantizer(8, False)
    q.quantize(torch.randn(10), torch.nn.Parameter(torch.tensor(0.1, dtype=torch.float64)), 0, True)
    crash = None
except Exception as e:  # TypeError
    crash = type(e).__name__
cases.append(dict(kind="asym_learnable_int_zp", raises=crash))

# ---------------------------------------------------------------------------
# 5. QuantizationManager sequence: calibrate (observe only) -> learn-init -> learnable fwd/bwd
# ---------------------------------------------------------------------------
mg_idx = 0
for bits, sym in ((4, True), (2, True), (8, False)):
    qm = QuantizationManager("UniformQuantizer", "MinMaxObserver", bits, sym, is_learning_scale=True)
    qm.is_observer_qparam, qm.is_learning_scale, qm.is_quantize = True, False, False
    g = torch.Generator().manual_seed(300 + mg_idx)
    xs = [torch.randn(4, 6, 5, 5, generator=g) * (0.5 + i) for i in range(3)]
    outs = [qm.quantize(x) for x in xs]
    identity_ok = all(torch.equal(o, x) for o, x in zip(outs, xs))
    calib = dict(min_val=float(qm.observer.min_val), max_val=float(qm.observer.max_val),
                 scale=float(qm.scale), zero_point=int(qm.zero_point),
                 mean_abs_x=list(map(float, qm.mean_abs_x)), mean_x=list(map(float, qm.mean_x)),
                 std=list(map(float, qm.std)))
    # observe + quantize in the same call
    qm.is_quantize = True
    x_oq = torch.randn(4, 6, 5, 5, generator=g)
    y_oq = qm.quantize(x_oq)
    oq = dict(scale=float(qm.scale), zero_point=int(qm.zero_point))
    # learn init + learnable step
    qm.is_learning_scale = True
    qm.init_scaling_factor_for_learning()
    init_scale = float(qm.scale)
    qm.make_learn_qparameter()
    key = f"mg{mg_idx}"
    mg_idx += 1
    x4 = torch.randn(4, 6, 5, 5, generator=g)
    gg = torch.randn(4, 6, 5, 5, generator=g)
    rec = dict(kind="manager_sequence", key=key, bits=bits, sym=sym, identity_ok=identity_ok,
               calib=calib, observe_quantize=oq, init_scale=init_scale,
               xs=[put(f"{key}_x{i}", x) for i, x in enumerate(xs)],
               x_oq=put(key + "_xoq", x_oq), y_oq=put(key + "_yoq", y_oq))
    try:
        xr = x4.clone().requires_grad_(True)
        y4 = qm.quantize(xr)
        y4.backward(gg)
        rec.update(x4=put(key + "_x4", x4), g4=put(key + "_g4", gg), y4=put(key + "_y4", y4),
                   gx4=put(key + "_gx4", xr.grad), scale_grad=float(qm.scale.grad),
                   scale_param_dtype=str(qm.scale.dtype))
    except Exception as e:
        rec.update(learn_raises=type(e).__name__)
    cases.append(rec)

# ---------------------------------------------------------------------------
# 6. Fused activation + activation fake-quant (K5): the fused layers run
#    F.relu / F.silu on the conv output (modules/fused.py:133) and then
#    quantize_out (quantizers/fake_quantize.py:49-50).  Gradients are w.r.t. the
#    pre-activation c (autograd through the activation).
# ---------------------------------------------------------------------------
import torch.nn.functional as F  # noqa: E402

act_idx = 0
for act in ("relu", "silu"):
    fn = F.relu if act == "relu" else F.silu
    for mode, sym, bits in (("observe", True, 8), ("observe", False, 8), ("observe", False, 4),
                            ("fixed", False, 8), ("fixed", True, 4),
                            ("learn", True, 8), ("learn", True, 4)):
        g = torch.Generator().manual_seed(500 + act_idx)
        c = torch.randn(4, 8, 6, 6, generator=g) * 1.5
        if mode == "fixed":   # specials: signed zeros, NaN, infinities, exact ties
            flat = c.view(-1)
            flat[:8] = torch.tensor([-0.0, 0.0, float("nan"), float("inf"), float("-inf"),
                                     -1e-40, 1e-40, 0.5])
        gg = torch.randn(c.shape, generator=torch.Generator().manual_seed(600 + act_idx))
        q = UniformQuantizer(bits, sym)
        cr = c.clone().requires_grad_(True)
        a = fn(cr)
        rec = dict(kind="act_fq", key=f"act{act_idx}", act=act, mode=mode, sym=sym, bits=bits)
        if mode == "observe":
            obs = MinMaxObserver(sym)          # num_bits 8 through the manager
            s_, z_ = obs.forward(a.detach())
            y = q.quantize(a, s_, z_, False)
            rec.update(scale=float(s_), zp=int(z_), min_val=float(obs.min_val), max_val=float(obs.max_val))
        elif mode == "fixed":
            s_, z_ = (0.05, 0) if sym else (0.03, 7)
            y = q.quantize(a, s_, z_, False)
            rec.update(scale=s_, zp=z_)
        else:
            scale = torch.nn.Parameter(torch.tensor(np.float64(0.04 if bits == 8 else 0.35)))
            y = q.quantize(a, scale, 0, True)
            rec.update(scale=float(scale.detach()), zp=0)
        y.backward(gg)
        key = rec["key"]
        rec.update(x=put(key + "_c", c), g=put(key + "_g", gg), y=put(key + "_y", y),
                   grad_x=put(key + "_gc", cr.grad))
        if mode == "learn":
            rec.update(scale_grad=float(scale.grad))
        cases.append(rec)
        act_idx += 1

# ---------------------------------------------------------------------------
# 7. LSQFakeQuantize (quantizers/lsq_module.py:73-166): the torch.ao-based LSQ module
#    with learnable fp32 scale_param / zero_point_param_float.  Calibrate with the
#    observer (3 batches), disable it, then one learnable fwd + bwd.  Per-channel
#    along axis 1 (the demo qconfig, lsq_module.py:509-517) and per-tensor; config_act
#    multiplies the gradient scale by 5000 (line 152).
# ---------------------------------------------------------------------------
from quantizers.lsq_module import LSQFakeQuantize  # noqa: E402

lsqm_idx = 0
for per_channel, config_act in ((True, False), (True, True), (False, False), (False, True)):
    torch.manual_seed(700 + lsqm_idx)
    if per_channel:
        fq = LSQFakeQuantize(learn_scale=True, config_act=config_act,
                             observer=torch.quantization.MovingAveragePerChannelMinMaxObserver,
                             quant_min=0, quant_max=255, dtype=torch.quint8,
                             qscheme=torch.per_channel_affine, reduce_range=False,
                             averaging_constant=0.01, ch_axis=1)
    else:
        fq = LSQFakeQuantize(learn_scale=True, config_act=config_act,
                             observer=torch.quantization.MovingAverageMinMaxObserver,
                             quant_min=0, quant_max=255, dtype=torch.quint8,
                             qscheme=torch.per_tensor_affine, reduce_range=False)
    shape = (4, 6, 9, 9)
    for _ in range(3):
        fq(torch.randn(shape) * 1.5 + 0.3)
    fq.disable_observer()
    x = torch.randn(shape) * 1.5 + 0.3
    gg = torch.randn(shape)
    xr = x.clone().requires_grad_(True)
    y = fq(xr)
    y.backward(gg)
    key = f"lsqm{lsqm_idx}"
    lsqm_idx += 1
    cases.append(dict(kind="lsq_fake_quantize", key=key, per_channel=per_channel, config_act=config_act,
                      qmin=0, qmax=255, x=put(key + "_x", x), g=put(key + "_g", gg), y=put(key + "_y", y),
                      grad_x=put(key + "_gx", xr.grad),
                      scale=put(key + "_scale", fq.scale_param.detach()),
                      zp=put(key + "_zp", fq.zero_point_param_float.detach()),
                      scale_grad=put(key + "_sgrad", fq.scale_param.grad),
                      zp_grad=put(key + "_zgrad", fq.zero_point_param_float.grad)))

# ---------------------------------------------------------------------------
# 8. Fused QAT layers (modules/fused.py:32-412): the BN fold at construction
#    (fused.py:100-108, 294-300) and one forward + backward through FakeQuantize.forward
#    (quantizers/fake_quantize.py:43-51) in the observe + quantize mode,
#    then -- symmetric layers -- the learnable mode after init_scaling_factor_for_learning
#    + make_learn_qparameter (qm.py:92-114).  The conv / linear itself is the host's
#    (MIOpen / hipBLASLt on the GPU box: not bitwise), so the intermediates around it
#    are recorded too: the fake-quantized weight and its gradient, the pre-activation
#    (the input of F.relu / F.silu, captured in modules.fused's namespace) and its
#    gradient.  Layers run in eval() (an unfolded BN uses its running statistics).
# ---------------------------------------------------------------------------
import copy  # noqa: E402

import torch.nn as nn  # noqa: E402
import modules.fused as RF  # noqa: E402


class _CaptureF:
    """Stand-in for modules.fused.F recording the pre-activation of F.relu / F.silu."""

    def __init__(self, real):
        self.real, self.seen = real, []

    def __getattr__(self, k):
        return getattr(self.real, k)

    def _cap(self, x):
        x.retain_grad()
        self.seen.append(x)

    def relu(self, x, *a, **k):
        self._cap(x)
        return self.real.relu(x, *a, **k)

    def silu(self, x, *a, **k):
        self._cap(x)
        return self.real.silu(x, *a, **k)


def _run_fused(m, x, g):
    """One forward + backward of a reference fused layer; returns the recorded tensors."""
    cap = _CaptureF(F)
    wq_seen, a_in = [], []
    orig_qw, orig_qa = m.quantize_weights, m.quantize_activation

    def qw(w):
        out = orig_qw(w)
        out.retain_grad()
        wq_seen.append(out)
        return out

    def qa(a):
        if a.requires_grad:
            a.retain_grad()
        a_in.append(a)
        return orig_qa(a)

    m.quantize_weights, m.quantize_activation = qw, qa
    RF.F = cap
    try:
        xr = x.clone().requires_grad_(True)
        y = m(xr)
        y.backward(g)
    finally:
        RF.F = F
        del m.quantize_weights, m.quantize_activation
    pre = cap.seen[0] if cap.seen else a_in[0]
    core = m.conv_fuse if hasattr(m, "conv_fuse") else m.linear_fuse
    out = dict(x=x, y=y, g=g, wq=wq_seen[0], grad_wq=wq_seen[0].grad, pre=pre, grad_pre=pre.grad,
               grad_x=xr.grad, grad_w=core.weight.grad)
    if core.bias is not None:
        out["grad_b"] = core.bias.grad
    core.weight.grad = None
    if core.bias is not None:
        core.bias.grad = None
    return out


def _qstate(qm):
    s, z = qm.scale, qm.zero_point
    return dict(scale=float(s.detach()) if isinstance(s, torch.Tensor) else float(s),
                zp=float(z.detach()) if isinstance(z, torch.Tensor) else float(z))


FUSED = [  # (class, conv?, bias, act, is_fuse_bn, w_sym, a_sym, bits_w, bits_a)
    ("ConvBnReLU", True, False, "relu", True, True, True, 4, 4),
    ("ConvBnReLU", True, True, "silu", True, True, True, 8, 8),
    ("ConvBnReLU", True, False, "relu", False, True, True, 2, 4),
    ("ConvBnReLU", True, True, "relu", True, False, False, 8, 8),
    ("ConvBn", True, True, None, True, True, True, 8, 4),
    ("ConvBn", True, False, None, False, True, True, 4, 8),
    ("ConvReLU", True, True, "relu", None, True, True, 4, 4),
    ("Conv", True, False, None, None, True, True, 8, 8),
    ("LinearBnReLU", False, True, "relu", True, True, True, 4, 4),
    ("LinearBnReLU", False, True, "silu", False, True, True, 8, 8),
    ("LinearBn", False, True, None, True, True, True, 2, 8),
]
fz_idx = 0
for cls_name, is_conv, bias, act, fuse_bn, w_sym, a_sym, bits_w, bits_a in FUSED:
    key = f"fz{fz_idx}"
    torch.manual_seed(800 + fz_idx)
    if is_conv:
        core = nn.Conv2d(6, 8, 3, padding=1, bias=bias)
        bn = nn.BatchNorm2d(8, eps=1e-3)
        xshape = (2, 6, 9, 9)
    else:
        core = nn.Linear(40, 24, bias=bias)
        bn = nn.BatchNorm1d(24)
        xshape = (5, 40)
    with torch.no_grad():
        bn.running_mean.uniform_(-0.3, 0.3)
        bn.running_var.uniform_(0.2, 3.0)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    act_mod = {"relu": nn.ReLU(), "silu": nn.SiLU(), None: None}[act]
    names = ("MinMaxObserver", "UniformQuantizer", "MinMaxObserver", "UniformQuantizer")
    cls = getattr(RF, cls_name)
    c0, b0 = copy.deepcopy(core), copy.deepcopy(bn)
    if cls_name in ("ConvBnReLU", "LinearBnReLU"):
        m = cls(c0, b0, act_mod, *names, w_sym, a_sym, fuse_bn, bits_w, bits_a)
    elif cls_name in ("ConvBn", "LinearBn"):
        m = cls(c0, b0, *names, w_sym, a_sym, fuse_bn, bits_w, bits_a)
    elif cls_name == "ConvReLU":
        m = cls(c0, act_mod, *names, w_sym, a_sym, bits_w, bits_a)
    else:
        m = cls(c0, *names, w_sym, a_sym, bits_w, bits_a)
    m.eval()
    lin = m.conv_fuse if is_conv else m.linear_fuse
    rec = dict(kind="fused_layer", key=key, cls=cls_name, conv=is_conv, bias=bias, act=act,
               is_fuse_bn=fuse_bn, w_sym=w_sym, a_sym=a_sym, bits_w=bits_w, bits_a=bits_a,
               bn_eps=float(bn.eps), core_w=put(key + "_cw", core.weight), bn_w=put(key + "_bnw", bn.weight),
               bn_b=put(key + "_bnb", bn.bias), bn_mean=put(key + "_bnm", bn.running_mean),
               bn_var=put(key + "_bnv", bn.running_var), fold_w=put(key + "_fw", lin.weight))
    if bias:
        rec["core_b"] = put(key + "_cb", core.bias)
    if lin.bias is not None:
        rec["fold_b"] = put(key + "_fb", lin.bias)
    gen = torch.Generator().manual_seed(900 + fz_idx)
    x = torch.randn(xshape, generator=gen)
    # observe + quantize mode (qm.py:65-90 with is_learning_scale False)
    for qm in (m.weight_quantizer, m.activation_quantizer):
        qm.is_learning_scale = False
    with torch.no_grad():
        yshape = m(x).shape
    for qm in (m.weight_quantizer, m.activation_quantizer):   # forget the shape probe
        qm.observer.min_val, qm.observer.max_val = 0, 0
        qm.mean_abs_x, qm.mean_x, qm.std = [], [], []
    g = torch.randn(yshape, generator=gen)
    r = _run_fused(m, x, g)
    rec["observe"] = dict({k: put(f"{key}_o_{k}", v) for k, v in r.items()},
                          wq_qp=_qstate(m.weight_quantizer), act_qp=_qstate(m.activation_quantizer))
    # learnable mode (symmetric layers; asymmetric + learnable raises in the reference, §0.5)
    if w_sym and a_sym:
        for qm in (m.weight_quantizer, m.activation_quantizer):
            qm.is_learning_scale = True
            qm.init_scaling_factor_for_learning()
            qm.make_learn_qparameter()
        inits = dict(w=float(m.weight_quantizer.scale.detach()), a=float(m.activation_quantizer.scale.detach()))
        x2 = torch.randn(xshape, generator=gen)
        g2 = torch.randn(yshape, generator=gen)
        r = _run_fused(m, x2, g2)
        rec["learn"] = dict({k: put(f"{key}_l_{k}", v) for k, v in r.items()}, init_scale_w=inits["w"],
                            init_scale_a=inits["a"],
                            scale_grad_w=float(m.weight_quantizer.scale.grad),
                            scale_grad_a=float(m.activation_quantizer.scale.grad))
    cases.append(rec)
    fz_idx += 1

# ---------------------------------------------------------------------------
# 9. fuse_modules_unified (modules/fuse.py:45-149, 254-277) on a toy model with a
#    FuseConfigManager (modules/fuse_config.py:57-149): which children fuse into which
#    class, with which quantizer settings.  The config lookup uses the CHILD name of the
#    first fused module (fuse.py:113-114), not its path: the pattern "stem" below
#    never matches, the pattern "^conv$" does.
# ---------------------------------------------------------------------------
from collections import OrderedDict  # noqa: E402

from modules.fuse import fuse_modules_unified  # noqa: E402
from modules.fuse_config import FuseConfig, FuseConfigManager  # noqa: E402


def toy_model():
    torch.manual_seed(1234)
    return nn.Sequential(OrderedDict(
        stem=nn.Sequential(OrderedDict(conv=nn.Conv2d(3, 8, 3, padding=1, bias=False),
                                       bn=nn.BatchNorm2d(8), act=nn.ReLU())),
        block=nn.Sequential(OrderedDict(conv1=nn.Conv2d(8, 8, 1), relu1=nn.SiLU(),
                                        conv2=nn.Conv2d(8, 16, 3, padding=1, bias=False),
                                        bn2=nn.BatchNorm2d(16))),
        tail=nn.Sequential(nn.Conv2d(16, 16, 3, padding=1), nn.ReLU(), nn.Conv2d(16, 4, 1)),
        head=nn.Sequential(OrderedDict(pool=nn.Flatten(), fc=nn.Linear(4 * 8 * 8, 10),
                                       bn=nn.BatchNorm1d(10), act=nn.ReLU())),
    ))


cm = FuseConfigManager(FuseConfig(bits_w=2, bits_a=4))
cm.add_layer_config("stem", FuseConfig(bits_w=8, bits_a=8))                    # path: never matches
cm.add_layer_config("^conv$", FuseConfig(bits_w=4, bits_a=4, w_symmetric=False))
cm.add_layer_config("conv2", FuseConfig(bits_w=6, bits_a=5, is_fuse_bn=False))
cm.add_layer_config("^0$", FuseConfig(bits_w=3, bits_a=3))
cm.add_layer_config("fc", FuseConfig(bits_w=8, bits_a=6, a_symmetric=False))
model = toy_model()
toy_sd = {k: v.clone() for k, v in model.state_dict().items()}
patterns = [["conv", "bn", "relu"], ["conv", "bn"], ["conv", "relu"], ["linear", "bn", "relu"],
            ["linear", "bn"], ["conv"], ["linear"]]
fused_model = fuse_modules_unified(model, patterns, is_trace=False, config_manager=cm)
struct = []
for name, mod in fused_model.named_modules():
    ent = dict(name=name, type=type(mod).__name__)
    if hasattr(mod, "weight_quantizer"):
        ent.update(bits_w=mod.bits_w, bits_a=mod.bits_a,
                   w_sym=mod.weight_quantizer.quantizer.symmetric,
                   a_sym=mod.activation_quantizer.quantizer.symmetric,
                   qw=type(mod.weight_quantizer.quantizer).__name__,
                   ow=type(mod.weight_quantizer.observer).__name__,
                   is_fuse_bn=getattr(mod, "is_fuse_bn", None), has_bn=hasattr(mod, "bn"),
                   is_relu=getattr(mod, "is_relu", None))
    struct.append(ent)
cases.append(dict(kind="fuse_structure", patterns=patterns, structure=struct,
                  configs={"default": dict(bits_w=2, bits_a=4), "stem": dict(bits_w=8, bits_a=8),
                           "^conv$": dict(bits_w=4, bits_a=4, w_symmetric=False),
                           "conv2": dict(bits_w=6, bits_a=5, is_fuse_bn=False),
                           "^0$": dict(bits_w=3, bits_a=3), "fc": dict(bits_w=8, bits_a=6, a_symmetric=False)},
                  state_dict={k: put("toy_" + k, v) for k, v in toy_sd.items()}))

np.savez_compressed(os.path.join(OUT, "fakequant_goldens.npz"), **arrays)
with open(os.path.join(OUT, "cases.json"), "w") as f:
    json.dump({"generator": "tests/golden/gen_goldens.py", "torch": torch.__version__,
               "reference": "tranngocduvnvp/VSIQuantization @ /root/reference", "cases": cases},
              f, indent=1)
print(f"{len(cases)} cases, {len(arrays)} arrays ->", OUT)
