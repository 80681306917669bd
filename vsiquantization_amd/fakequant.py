"""torch-facing fake-quant ops over the HIP C ABI (CPU tensors: the native host loops of
host.py, never the oracle).

Each op here is one (or two) kernel launches on the tensor's current HIP
stream, no host synchronisation, and is the MI355X replacement of one chain of
eager torch ops in the reference:

  fake_quant               quantizers/uniform.py:54-55,95   (K1)
  observe_tensor           observers/minmax.py:32-88 + quantization_manager.py:66-68 (K2)
  per_channel_observe_fq   per-channel MinMax + UniformQuantizer (K3)
  FakeQuantFixedFn         autograd of uniform.py:55,95 with fixed qparams (STE)
  FakeQuantLearnFn         autograd of uniform.py:47-56 (LSQ: ScaleGradient, STE) (K4)
  FakeQuantLearnMultiFn    FakeQuantLearnFn over many tensors in one launch each way
  observe_parts/fold_parts deferred-calibration observer (K2p) and its one-launch fold
  observe_parts_out        K2p that also writes act(x): a fused layer's calibration forward (K2o)

Every op takes an optional ``act`` ("relu" / "silu", K5): the op is then applied
to act(x) without materializing it -- the fused layers' F.relu / F.silu before
quantize_out (modules/fused.py:124-134, quantizers/fake_quantize.py:49-50) -- and
the backward ops return the gradient with respect to the pre-activation x.
"""
from __future__ import annotations

import ctypes
import numbers

import numpy as np
import torch

from . import _hip as H
from . import host as _host


# --------------------------------------------------------------------------- scalars
def qden(symmetric: bool, num_bits: int, eps: float) -> float:
    """Denominator of minmax.py:72 / :75, evaluated with Python floats like the reference."""
    return (2 ** (num_bits - 1) - 1 + eps) if symmetric else (2 ** num_bits - 1 + eps)


def _as_f64_device(t: torch.Tensor, device) -> torch.Tensor:
    t = t.detach()
    if t.numel() != 1:
        raise ValueError(f"expected a scalar (1-element) qparam tensor, got shape {tuple(t.shape)}")
    if t.device != device:
        t = t.to(device, non_blocking=True)
    if t.dtype != torch.float64:
        t = t.to(torch.float64)
    return t.contiguous()


def scalar_source(v, device):
    """Resolve a scale / zero-point argument into (device f64 tensor | None, host float).

    Python numbers and CPU tensors are read on the host (no GPU sync); CUDA
    tensors are passed by pointer so the kernel reads the current value."""
    if isinstance(v, torch.Tensor):
        if v.device.type == "cuda":
            return _as_f64_device(v, device), 0.0
        return None, float(v.detach().reshape(()).item())
    if isinstance(v, (numbers.Real, np.floating, np.integer)):
        return None, float(v)
    raise TypeError(f"unsupported qparam type {type(v).__name__}")


def _i64(n):
    return H.c_i64(int(n))


# --------------------------------------------------------------------------- forward (K1)
def fake_quant(x: torch.Tensor, scale, zero_point, qmin: int, qmax: int, *, zp_round: bool = False,
               qp: torch.Tensor | None = None, want_mask: bool = False, want_codes: bool = False,
               discrete: bool = False, act=None):
    """y = (clamp(rint(x/s + zp), qmin, qmax) - zp) * s  (uniform.py:55,95), fp32, bit-exact.

    qp: optional observer record (f64[QP_LEN] on x.device) used instead of scale/zero_point.
    discrete: return the integer-valued fp32 codes in y instead (discreate_tensor).
    Returns (y, mask|None, codes|None); codes int8 (qmin<0) or uint8.  A CPU tensor takes
    the native host path (host.py; its mask is one byte per element)."""
    if _host.is_host(x):
        return _host.fake_quant(x, scale, zero_point, qmin, qmax, zp_round=zp_round, qp=qp, want_mask=want_mask,
                                want_codes=want_codes, discrete=discrete, act=act)
    x = H.require_device_f32(x)
    dev = x.device
    y = torch.empty_like(x)
    mask = H.mask_buffer(1, x.numel(), dev) if want_mask else None
    codes = None
    if want_codes:
        codes = torch.empty(x.shape, dtype=torch.int8 if qmin < 0 else torch.uint8, device=dev)
    if qp is not None:
        sd, sh, zd, zh = None, 0.0, None, 0.0
    else:
        sd, sh = scalar_source(scale, dev)
        zd, zh = scalar_source(zero_point, dev)
    rc = H.lib().vsiq_act_fq_fwd_f32(H.ptr(x), H.ptr(y), H.ptr(codes), H.ptr(mask), _i64(x.numel()),
                                     H.act_code(act), H.ptr(qp), H.ptr(sd), sh, H.ptr(zd), zh,
                                     int(bool(zp_round)), int(bool(discrete)), int(qmin), int(qmax),
                                     H.stream_of(dev))
    H.check(rc, "vsiq_act_fq_fwd_f32")
    return y, mask, codes


def ste_backward(g: torch.Tensor, mask: torch.Tensor, scale, rowlen: int = 0, *, pre=None,
                 act=None) -> torch.Tensor:
    """gx = (mask ? g*s : 0) / s  — autograd of uniform.py:55,95 with a fixed scale;
    with ``act``, the activation's backward at the pre-activation ``pre`` follows."""
    g = H.require_device_f32(g, "grad_output")
    a = H.act_code(act)
    if a != H.ACT_NONE:
        pre = H.require_device_f32(pre, "pre-activation")
        if pre.shape != g.shape:
            raise ValueError(f"pre-activation shape {tuple(pre.shape)} != grad shape {tuple(g.shape)}")
    dev = g.device
    gx = torch.empty_like(g)
    if isinstance(scale, torch.Tensor) and scale.device.type == "cuda" and scale.numel() > 1:
        sd, sh = scale.detach().to(torch.float64).contiguous(), 0.0
    else:
        sd, sh = scalar_source(scale, dev)
        rowlen = 0
    rc = H.lib().vsiq_act_ste_bwd_f32(H.ptr(g), H.ptr(mask), H.ptr(pre if a else None), H.ptr(gx),
                                      _i64(g.numel()), a, H.ptr(sd), _i64(rowlen), sh, H.stream_of(dev))
    H.check(rc, "vsiq_act_ste_bwd_f32")
    return gx


# --------------------------------------------------------------------------- activation alone
class ActivationFn(torch.autograd.Function):
    """act(x) on its own (vsiq_act_fwd_f32 / vsiq_act_bwd_f32): the fused layers' F.silu
    (modules/fused.py:133) where its output is not fake-quantized in the same pass
    (calibration forwards), bit for bit as torch's CPU kernel computes it."""

    @staticmethod
    def forward(ctx, x, act):
        x = H.require_device_f32(x)
        code = H.act_code(act)
        y = torch.empty_like(x)
        H.check(H.lib().vsiq_act_fwd_f32(H.ptr(x), H.ptr(y), _i64(x.numel()), code, H.stream_of(x.device)),
                "vsiq_act_fwd_f32")
        ctx.code = code
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        g = H.require_device_f32(g, "grad_output")
        gx = torch.empty_like(x)
        H.check(H.lib().vsiq_act_bwd_f32(H.ptr(g), H.ptr(x), H.ptr(gx), _i64(x.numel()), ctx.code,
                                         H.stream_of(x.device)), "vsiq_act_bwd_f32")
        return gx, None


def activation(x, act):
    """The fused layers' F.relu / F.silu (modules/fused.py:133) as the reference computes
    them on its CPU tensors: a CUDA fp32 tensor goes through ActivationFn (torch's HIP silu
    uses another exp, and its HIP relu turns -0.0 into +0.0 where the CPU kernel keeps
    -0.0); anything else is torch's own CPU op, i.e. the reference's."""
    if act not in ("relu", "silu"):
        raise ValueError(f"unsupported fused activation {act!r} ('relu' or 'silu')")
    if isinstance(x, torch.Tensor) and x.device.type == "cuda" and x.dtype == torch.float32:
        return ActivationFn.apply(x, act)
    return torch.nn.functional.relu(x) if act == "relu" else torch.nn.functional.silu(x)


class FakeQuantFixedFn(torch.autograd.Function):
    """Fixed-qparam fake quant with the reference's STE gradient (x only)."""

    @staticmethod
    def forward(ctx, x, scale, zero_point, qmin, qmax, qp, act=None):
        y, mask, _ = fake_quant(x, scale, zero_point, qmin, qmax, qp=qp, want_mask=True, act=act)
        ctx.act = act
        if H.act_code(act) != H.ACT_NONE:
            ctx.save_for_backward(mask, x)
        else:
            ctx.save_for_backward(mask)
        if qp is not None:
            ctx.scale = qp[H.QP_SCALE:H.QP_SCALE + 1]
        else:
            ctx.scale = scale.detach() if isinstance(scale, torch.Tensor) else scale
        return y

    @staticmethod
    def backward(ctx, gy):
        saved = ctx.saved_tensors
        pre = saved[1] if len(saved) > 1 else None
        gx = ste_backward(gy.contiguous(), saved[0], ctx.scale, pre=pre, act=ctx.act)
        return gx, None, None, None, None, None, None


def _qarg(v):
    """A scale / zero-point argument as (tensor | None, host float) for the C++ nodes:
    tensors go through as tensors (the node reads a CUDA one by pointer and keeps the
    autograd edge of a learnable one), numbers as host floats."""
    if isinstance(v, torch.Tensor):
        return v, 0.0
    if isinstance(v, (numbers.Real, np.floating, np.integer)):
        return None, float(v)
    raise TypeError(f"unsupported qparam type {type(v).__name__}")


def fake_quant_fixed(x, scale, zero_point, qmin, qmax, qp=None, act=None):
    """Fixed-qparam fake quant; with a gradient-requiring x, the STE backward is attached
    (C++ node of _vsiq_torch.so, or FakeQuantFixedFn with VSIQ_TORCH_EXT=0).  CPU tensors:
    the native host path (host.py)."""
    if _host.is_host(x):
        return _host.fake_quant_fixed(x, scale, zero_point, qmin, qmax, qp=qp, act=act)
    if x.requires_grad and torch.is_grad_enabled():
        if H.torch_ext_enabled():
            x = H.require_device_f32(x)
            st, sh = _qarg(scale) if qp is None else (None, 0.0)
            zt, zh = _qarg(zero_point) if qp is None else (None, 0.0)
            return H.torch_ext().fq_fixed(x, st, sh, zt, zh, int(qmin), int(qmax), qp, H.act_code(act))
        return FakeQuantFixedFn.apply(x, scale, zero_point, qmin, qmax, qp, act)
    return fake_quant(x, scale, zero_point, qmin, qmax, qp=qp, act=act)[0]


def fake_quant_learn(x, scale, zero_point, qmin, qmax, gscale, learn_zp, act=None):
    """Learnable fake quant (uniform.py:47-56): K1/K5 forward, K4 backward with the
    ScaleGradient factor ``gscale`` (C++ node of _vsiq_torch.so, or FakeQuantLearnFn
    with VSIQ_TORCH_EXT=0).  CPU tensors: the native host path (host.py)."""
    if _host.is_host(x):
        return _host.fake_quant_learn(x, scale, zero_point, qmin, qmax, gscale, learn_zp, act)
    if H.torch_ext_enabled() and learn_zp != 2:   # the C++ node takes its K4 workspace from its own cache
        x = H.require_device_f32(x)
        st, sh = _qarg(scale)
        zt, zh = _qarg(zero_point)
        return H.torch_ext().fq_learn(x, st, sh, zt, zh, int(qmin), int(qmax), float(gscale), bool(learn_zp),
                                      H.act_code(act))
    return FakeQuantLearnFn.apply(x, scale, zero_point, qmin, qmax, gscale, learn_zp, act)


# --------------------------------------------------------------------------- learnable (K4)
def lsq_backward(g, x, scale, zero_point, qmin, qmax, gscale, learn_zp, act=None):
    """K4: (grad_x, f64[2] {grad_scale, grad_zp}); with ``act``, x is the pre-activation
    and grad_x goes through the activation's backward."""
    g = H.require_device_f32(g, "grad_output")
    dev = g.device
    gx = torch.empty_like(g)
    grads = torch.empty(2, dtype=torch.float64, device=dev)
    sd, sh = scalar_source(scale, dev)
    zd, zh = scalar_source(zero_point, dev)
    w = H.workspace(dev, g.numel())
    rc = H.lib().vsiq_act_lsq_bwd_f32(H.ptr(g), H.ptr(x), H.ptr(gx), _i64(g.numel()), H.act_code(act),
                                      H.ptr(sd), sh, H.ptr(zd), zh, int(learn_zp), int(qmin),
                                      int(qmax), float(gscale), H.ptr(grads), H.ptr(w.ws),
                                      _i64(w.ws_len), H.ptr(w.counter), H.stream_of(dev))
    H.check(rc, "vsiq_act_lsq_bwd_f32")
    return gx, grads


class FakeQuantLearnFn(torch.autograd.Function):
    """Learnable-scale (and, asymmetric, learnable zero-point) fake quant.

    Forward = uniform.py:47-56; backward = the reference's autograd graph in closed
    form (ScaleGradient x gscale on scale and zp, ClampBackward1 mask, STE)."""

    @staticmethod
    def forward(ctx, x, scale, zero_point, qmin, qmax, gscale, learn_zp, act=None):
        x = H.require_device_f32(x)
        y, _, _ = fake_quant(x, scale, zero_point, qmin, qmax, zp_round=learn_zp == 1, act=act)
        ctx.save_for_backward(x)
        ctx.scale, ctx.zp = scale, zero_point
        ctx.args = (qmin, qmax, gscale, learn_zp, act)
        return y

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        qmin, qmax, gscale, learn_zp, act = ctx.args
        s, z = ctx.scale, ctx.zp
        gx, grads = lsq_backward(gy.contiguous(), x, s, z, qmin, qmax, gscale, learn_zp, act=act)
        gs = gz = None
        if isinstance(s, torch.Tensor) and ctx.needs_input_grad[1]:
            gs = grads[0].to(device=s.device, dtype=s.dtype).reshape(s.shape)
        if learn_zp and isinstance(z, torch.Tensor) and ctx.needs_input_grad[2]:
            gz = grads[1].to(device=z.device, dtype=z.dtype).reshape(z.shape)
        return gx, gs, gz, None, None, None, None, None


# --------------------------------------------------------------------------- multi-tensor learnable
class LsqSpec:
    """One tensor of a multi-tensor learnable fake quant: qmin/qmax, the ScaleGradient
    factor, whether the zero point is learned, and scale / zero point as device f64
    tensors or host numbers (exactly the arguments of FakeQuantLearnFn)."""

    __slots__ = ("scale", "zero_point", "qmin", "qmax", "gscale", "learn_zp")

    def __init__(self, scale, zero_point, qmin, qmax, gscale, learn_zp):
        self.scale, self.zero_point = scale, zero_point
        self.qmin, self.qmax, self.gscale, self.learn_zp = int(qmin), int(qmax), float(gscale), bool(learn_zp)


def _lsq_descs(specs, xs, ys=None, gs=None, gxs=None, grads=None):
    """ctypes array of vsiq_lsq_tensor + the device f64 scale/zp copies it points to."""
    arr = (H.LsqTensor * len(specs))()
    keep = []
    for i, (sp, x) in enumerate(zip(specs, xs)):
        d = arr[i]
        sd, sh = scalar_source(sp.scale, x.device)
        zd, zh = scalar_source(sp.zero_point, x.device)
        keep += [sd, zd]
        d.x = x.data_ptr()
        d.y = ys[i].data_ptr() if ys is not None else None
        d.g = gs[i].data_ptr() if gs is not None else None
        d.gx = gxs[i].data_ptr() if gxs is not None else None
        d.scale_dev = sd.data_ptr() if sd is not None else None
        d.zp_dev = zd.data_ptr() if zd is not None else None
        d.grad_out = grads[i].data_ptr() if grads is not None else None
        d.n, d.scale_host, d.zp_host, d.gscale = x.numel(), sh, zh, sp.gscale
        d.qmin, d.qmax, d.zp_learn = sp.qmin, sp.qmax, int(sp.learn_zp)
    return arr, keep


class FakeQuantLearnMultiFn(torch.autograd.Function):
    """FakeQuantLearnFn over many tensors at once (k_multi.hip): one forward launch and
    one backward launch for all of them; per tensor bit-identical to FakeQuantLearnFn.

    apply(specs, *xs, *scale_and_zp_tensors): the learnable tensors referenced by the
    specs are passed again as inputs so autograd routes their gradients."""

    @staticmethod
    def forward(ctx, specs, *inputs):
        k = len(specs)
        xs = [H.require_device_f32(x) for x in inputs[:k]]
        if not xs:
            return ()
        dev = xs[0].device
        if any(x.device != dev for x in xs):
            raise ValueError("multi-tensor fake quant: all tensors must be on one device")
        ys = [torch.empty_like(x) for x in xs]
        arr, keep = _lsq_descs(specs, xs, ys=ys)
        H.check(H.lib().vsiq_lsq_fwd_multi_f32(ctypes.cast(arr, ctypes.c_void_p), k, H.stream_of(dev)),
                "vsiq_lsq_fwd_multi_f32")
        ctx.save_for_backward(*xs)
        ctx.specs = specs
        ctx.params = inputs[k:]
        return tuple(ys)

    @staticmethod
    def backward(ctx, *gys):
        xs = ctx.saved_tensors
        specs = ctx.specs
        k = len(specs)
        dev = xs[0].device
        gs = [H.require_device_f32(g, "grad_output") for g in gys]
        gxs = [torch.empty_like(x) for x in xs]
        grads = torch.empty(k, 2, dtype=torch.float64, device=dev)
        arr, keep = _lsq_descs(specs, xs, gs=gs, gxs=gxs, grads=grads)
        p = ctypes.cast(arr, ctypes.c_void_p)
        need = int(H.lib().vsiq_lsq_multi_workspace_doubles(p, k))
        H.check(need if need < 0 else 0, "vsiq_lsq_multi_workspace_doubles")
        w = H.workspace(dev).reserve_doubles(need)
        rc = H.lib().vsiq_lsq_bwd_multi_f32(p, k, H.ptr(w.ws), _i64(w.ws_len), H.ptr(w.counter),
                                            H.stream_of(dev))
        H.check(rc, "vsiq_lsq_bwd_multi_f32")
        # gradients of the learnable scale / zero-point tensors, in input order
        out = []
        j = k
        for i, sp in enumerate(specs):
            for col, v, learn in ((0, sp.scale, True), (1, sp.zero_point, sp.learn_zp)):
                if isinstance(v, torch.Tensor) and v.requires_grad:
                    g = None
                    if learn and ctx.needs_input_grad[1 + j]:
                        g = grads[i, col].to(device=v.device, dtype=v.dtype).reshape(v.shape)
                    out.append(g)
                    j += 1
        return (None, *gxs, *out)


def _ext_qarg(v):
    """(CUDA tensor | None, host float) of a scale / zero point for the C++ K7 node, or
    None when only the Python Function routes it (a gradient-requiring host tensor)."""
    if isinstance(v, torch.Tensor):
        if v.device.type == "cuda":
            return v, 0.0
        if v.requires_grad:
            return None
        return None, float(v.detach().reshape(()).item())
    return None, float(v)


def lsq_fake_quant_multi(xs, specs):
    """Learnable fake quant of every x in ``xs`` with its LsqSpec, in one launch each way
    (the C++ node LsqMultiBackward of _vsiq_torch.so, or FakeQuantLearnMultiFn with
    VSIQ_TORCH_EXT=0)."""
    if H.torch_ext_enabled() and xs:
        qs = [(_ext_qarg(sp.scale), _ext_qarg(sp.zero_point)) for sp in specs]
        if all(a is not None and b is not None for a, b in qs):
            xs = [H.require_device_f32(x) for x in xs]
            return tuple(H.torch_ext().lsq_multi(xs, [a[0] for a, _ in qs], [a[1] for a, _ in qs],
                                                 [b[0] for _, b in qs], [b[1] for _, b in qs],
                                                 [sp.qmin for sp in specs], [sp.qmax for sp in specs],
                                                 [sp.gscale for sp in specs], [sp.learn_zp for sp in specs]))
    params = [v for sp in specs for v in (sp.scale, sp.zero_point)
              if isinstance(v, torch.Tensor) and v.requires_grad]
    return FakeQuantLearnMultiFn.apply(tuple(specs), *xs, *params)


# --------------------------------------------------------------------------- observer (K2)
def observe_tensor(x: torch.Tensor, *, symmetric: bool, num_bits: int = 8, eps: float = 1e-8,
                   run_minmax: torch.Tensor | None = None, want_qp: bool = True,
                   want_stats: bool = True, act=None):
    """One pass over x: min/max/NaN/sums -> running state update -> f64 qparams (no sync).

    Returns (qp f64[QP_LEN] | None, stats f64[ST_LEN] | None).  CPU tensors: the native
    host path (host.py; run_minmax a CPU fp32[2])."""
    if _host.is_host(x):
        return _host.observe_tensor(x, symmetric=symmetric, num_bits=num_bits, eps=eps, run_minmax=run_minmax,
                                    want_qp=want_qp, want_stats=want_stats, act=act)
    x = H.require_device_f32(x)
    if x.numel() == 0:
        raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0.")
    dev = x.device
    qp = torch.empty(H.QP_LEN, dtype=torch.float64, device=dev) if want_qp else None
    st = torch.empty(H.ST_LEN, dtype=torch.float64, device=dev) if want_stats else None
    w = H.workspace(dev, x.numel())
    rc = H.lib().vsiq_act_observe_f32(H.ptr(x), _i64(x.numel()), H.act_code(act), H.ptr(st),
                                      H.ptr(run_minmax), H.ptr(qp), int(bool(symmetric)),
                                      qden(symmetric, num_bits, eps), float(eps), H.ptr(w.ws),
                                      _i64(w.ws_len), H.ptr(w.counter), H.stream_of(dev))
    H.check(rc, "vsiq_act_observe_f32")
    return qp, st


# K8 (one workgroup holds the tensor) up to here; K9 above: through the API K8 is
# 10.9-12.1 us against 17.9-18.2 us for K2 + K1 at 432-16384 elements, but its GPU time
# grows past K2 + K1's ~9 us above ~16K elements (65536: 16.2 us; tools/exp/k8_bench.py).
_K8_ELEMS = 16384


def observe_fq_max_elems() -> int:
    """Largest tensor observe_fake_quant takes in ONE launch (K8: one workgroup holds it
    in registers)."""
    return int(H.lib().vsiq_observe_fq_max_elems())


def observe_fq_parts_max_elems() -> int:
    """Largest tensor observe_fake_quant takes on the K2p + fold-in-every-workgroup path (K9)."""
    return int(H.lib().vsiq_observe_fq_parts_max_elems())


def observe_fake_quant(x: torch.Tensor, *, symmetric: bool, num_bits: int = 8, eps: float = 1e-8,
                       qmin: int, qmax: int, run_minmax: torch.Tensor | None = None, act=None,
                       want_mask: bool = False, want_codes: bool = False, parts: bool | None = None):
    """Per-tensor observe (running update, f64 qparams, stats) + fake quant of one tensor
    -- observe_tensor + fake_quant(qp=...) fused.  K8 (one launch, one workgroup) up to
    ``_K8_ELEMS`` elements, K9 (K2p records + a fake-quant launch whose every workgroup
    folds them; no arrival chain) above, up to observe_fq_parts_max_elems().  ``parts``:
    False forces K8, True / "k9" K9, "k10" the one-launch K10 (K2p records, a grid
    barrier, every workgroup folds them and quantizes from registers; the same bits as K9,
    and no faster on MI355X: the barrier costs what the second launch does).
    Returns (y, qp f64[QP_LEN], stats f64[ST_LEN], mask | None, codes | None)."""
    x = H.require_device_f32(x)
    n = x.numel()
    if n == 0:
        raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0.")
    dev = x.device
    y = torch.empty_like(x)
    qp = torch.empty(H.QP_LEN, dtype=torch.float64, device=dev)
    st = torch.empty(H.ST_LEN, dtype=torch.float64, device=dev)
    mask = H.mask_buffer(1, n, dev) if want_mask else None
    codes = torch.empty(x.shape, dtype=torch.int8 if qmin < 0 else torch.uint8, device=dev) if want_codes else None
    if parts is None:
        parts = n > _K8_ELEMS
    if parts == "k10":
        w = H.workspace(dev, n)
        rc = H.lib().vsiq_act_observe_fq_grid_f32(H.ptr(x), H.ptr(y), H.ptr(codes), H.ptr(mask), _i64(n),
                                                  H.act_code(act), H.ptr(st), H.ptr(run_minmax), H.ptr(qp),
                                                  int(bool(symmetric)), qden(symmetric, num_bits, eps), float(eps),
                                                  int(qmin), int(qmax), H.ptr(w.ws), _i64(w.ws_len),
                                                  H.ptr(w.counter), H.stream_of(dev))
        H.check(rc, "vsiq_act_observe_fq_grid_f32")
        # a workgroup that timed out at the grid barrier wrote NaN and counted itself: fail
        # loudly (one host sync; K10 is an opt-in measurement path; not checkable while the
        # stream is being captured into a HIP graph -- the next eager call reports it)
        err = w.counter[H.COUNTER_GRID_ERRORS:H.COUNTER_GRID_ERRORS + 1]
        if not torch.cuda.is_current_stream_capturing() and int(err.item()):
            err.zero_()
            raise H.VsiqError("vsiq_act_observe_fq_grid_f32: grid barrier timed out (the grid was not "
                              "co-resident); the outputs of the timed-out workgroups are NaN")
    elif parts:   # True / "k9"
        w = H.workspace(dev, n)
        rc = H.lib().vsiq_act_observe_fq_parts_f32(H.ptr(x), H.ptr(y), H.ptr(codes), H.ptr(mask), _i64(n),
                                                   H.act_code(act), H.ptr(st), H.ptr(run_minmax), H.ptr(qp),
                                                   int(bool(symmetric)), qden(symmetric, num_bits, eps), float(eps),
                                                   int(qmin), int(qmax), H.ptr(w.ws), _i64(w.ws_len),
                                                   H.stream_of(dev))
        H.check(rc, "vsiq_act_observe_fq_parts_f32")
    else:
        rc = H.lib().vsiq_act_observe_fq_f32(H.ptr(x), H.ptr(y), H.ptr(codes), H.ptr(mask), _i64(n),
                                             H.act_code(act), H.ptr(st), H.ptr(run_minmax), H.ptr(qp),
                                             int(bool(symmetric)), qden(symmetric, num_bits, eps), float(eps),
                                             int(qmin), int(qmax), H.stream_of(dev))
        H.check(rc, "vsiq_act_observe_fq_f32")
    return y, qp, st, mask, codes


class ObserveFakeQuantFn(torch.autograd.Function):
    """K8 forward (observe + fake quant in one launch) with the reference's STE gradient
    at fp32(scale) of this call (the FakeQuantFixedFn backward)."""

    @staticmethod
    def forward(ctx, x, symmetric, num_bits, eps, qmin, qmax, run_minmax, act):
        y, qp, st, mask, _ = observe_fake_quant(x, symmetric=symmetric, num_bits=num_bits, eps=eps, qmin=qmin,
                                                qmax=qmax, run_minmax=run_minmax, act=act, want_mask=True)
        ctx.act = act
        ctx.save_for_backward(mask, x) if H.act_code(act) != H.ACT_NONE else ctx.save_for_backward(mask)
        ctx.scale = qp[H.QP_SCALE:H.QP_SCALE + 1]
        ctx.mark_non_differentiable(qp, st)
        return y, qp, st

    @staticmethod
    def backward(ctx, gy, _gqp, _gst):
        saved = ctx.saved_tensors
        pre = saved[1] if len(saved) > 1 else None
        gx = ste_backward(gy.contiguous(), saved[0], ctx.scale, pre=pre, act=ctx.act)
        return gx, None, None, None, None, None, None, None


def part_slot_doubles(n: int | None = None) -> int:
    """Doubles of one deferred-observer slot for n elements (K2p records x VSIQ_PART_LEN);
    n None: a slot that fits any n."""
    if n is None:
        return H.PART_MAX_RECORDS * H.PART_LEN
    r = int(H.lib().vsiq_observe_part_records(_i64(n)))
    H.check(r if r < 0 else 0, "vsiq_observe_part_records")
    return r * H.PART_LEN


def part_out_slot_doubles(n: int) -> int:
    """Doubles of one K2o slot for n elements (vsiq_observe_part_out_records(n) x
    VSIQ_PART_LEN; one record per workgroup of the one-shot pass)."""
    r = int(H.lib().vsiq_observe_part_out_records(_i64(n)))
    H.check(r if r < 0 else 0, "vsiq_observe_part_out_records")
    return r * H.PART_LEN


def observe_parts(x: torch.Tensor, out: torch.Tensor | None = None, act=None) -> torch.Tensor:
    """Deferred observer pass (K2p): the per-wave partial records of act(x) into
    ``out`` (f64, >= part_slot_doubles(numel) entries; allocated when None), no fold,
    no running update.  Fold with ``fold_parts``."""
    x = H.require_device_f32(x)
    if x.numel() == 0:
        raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0.")
    need = part_slot_doubles(x.numel())
    if out is None:
        out = torch.empty(need, dtype=torch.float64, device=x.device)
    elif out.dtype != torch.float64 or out.device != x.device or not out.is_contiguous():
        raise ValueError("observe_parts: out must be a contiguous float64 tensor on x's device")
    rc = H.lib().vsiq_act_observe_part_f32(H.ptr(x), _i64(x.numel()), H.act_code(act), H.ptr(out),
                                           _i64(out.numel()), H.stream_of(x.device))
    H.check(rc, "vsiq_act_observe_part_f32")
    return out


def observe_parts_out(x: torch.Tensor, act, out: torch.Tensor | None = None):
    """K2o: y = act(x) and the deferred observer records of act(x) (observe_parts) in ONE
    pass -- a fused layer's calibration forward (modules/fused.py:133 + minmax.py:42-43).
    ``out`` holds >= part_out_slot_doubles(numel) doubles (records in observe_parts'
    format, one per workgroup; fold with ``fold_parts``).  Returns (y, out)."""
    x = H.require_device_f32(x)
    if x.numel() == 0:
        raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0.")
    need = part_out_slot_doubles(x.numel())
    if out is None:
        out = torch.empty(need, dtype=torch.float64, device=x.device)
    elif out.dtype != torch.float64 or out.device != x.device or not out.is_contiguous() or out.numel() < need:
        raise ValueError("observe_parts_out: out must be a contiguous float64 tensor on x's device")
    y = torch.empty_like(x)
    rc = H.lib().vsiq_act_observe_part_out_f32(H.ptr(x), H.ptr(y), _i64(x.numel()), H.act_code(act), H.ptr(out),
                                               _i64(out.numel()), H.stream_of(x.device))
    H.check(rc, "vsiq_act_observe_part_out_f32")
    return y, out


def observe_parts_multi(xs, outs, act=None) -> list:
    """K2m: the deferred observer pass (observe_parts) of every x in ``xs`` into its slot
    in ``outs`` (None: allocated) in one launch per 32 tensors, on the current stream of
    the first x's device.  Records bit-identical to one observe_parts call per x."""
    if not xs:
        return []
    dev = xs[0].device
    arr = (H.PartTensor * len(xs))()
    res = []
    for i, x in enumerate(xs):
        x = H.require_device_f32(x)
        if x.device != dev:
            raise ValueError("observe_parts_multi: all tensors must be on one device")
        if x.numel() == 0:
            raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0.")
        out = outs[i] if outs is not None else None
        need = part_slot_doubles(x.numel())
        if out is None:
            out = torch.empty(need, dtype=torch.float64, device=dev)
        elif out.dtype != torch.float64 or out.device != dev or not out.is_contiguous():
            raise ValueError("observe_parts_multi: slots must be contiguous float64 tensors on x's device")
        arr[i] = H.PartTensor(x.data_ptr(), x.numel(), out.data_ptr(), out.numel())
        res.append(out)
    rc = H.lib().vsiq_act_observe_part_multi_f32(arr, len(xs), H.act_code(act), H.stream_of(dev))
    H.check(rc, "vsiq_act_observe_part_multi_f32")
    return res


def fold_parts(parts: torch.Tensor) -> torch.Tensor:
    """Fold deferred observer slots ``parts`` [calls, stride] (f64, one call per row) into
    stats records f64 [calls, ST_LEN] in one launch."""
    if parts.dim() != 2 or parts.dtype != torch.float64 or not parts.is_cuda or not parts.is_contiguous():
        raise ValueError("fold_parts: parts must be a contiguous CUDA float64 [calls, stride] tensor")
    st = torch.empty(parts.shape[0], H.ST_LEN, dtype=torch.float64, device=parts.device)
    rc = H.lib().vsiq_observe_fold_parts(H.ptr(parts), _i64(parts.shape[0]), _i64(parts.shape[1]),
                                         H.ptr(st), H.stream_of(parts.device))
    H.check(rc, "vsiq_observe_fold_parts")
    return st


def observe_finalize(stats: torch.Tensor, run_minmax, *, symmetric, num_bits=8, eps=1e-8):
    """Running update + qparams from an (all-reduced) stats record; returns qp f64[QP_LEN]."""
    dev = stats.device
    qp = torch.empty(H.QP_LEN, dtype=torch.float64, device=dev)
    rc = H.lib().vsiq_observe_finalize(H.ptr(stats), H.ptr(run_minmax), H.ptr(qp), int(bool(symmetric)),
                                       qden(symmetric, num_bits, eps), float(eps), H.stream_of(dev))
    H.check(rc, "vsiq_observe_finalize")
    return qp


# --------------------------------------------------------------------------- per-channel (K3)
def per_channel_observe_fq(x: torch.Tensor, *, symmetric: bool, qmin: int, qmax: int,
                           obs_bits: int = 8, eps: float = 1e-8, run_min=None, run_max=None,
                           quantize: bool = True, want_mask: bool = False, want_codes: bool = False,
                           want_row_stats: bool = False):
    """Fused per-channel (axis 0) MinMax observe + f64 qparams + fake quant, one pass (K3).

    quantize=False observes only (state, qparams, stats; y is None).
    Returns dict(y, scale f64[C], zp f64[C], run_min, run_max, mask, codes, row_stats f64[C,3])."""
    x = H.require_device_f32(x)
    dev = x.device
    C = x.shape[0] if x.dim() > 0 else 1
    rowlen = x.numel() // max(C, 1)
    if run_min is None or run_max is None:   # fresh observer state 0/0 (minmax.py:28-29), one fill
        state = torch.zeros(2, C, dtype=torch.float32, device=dev)
        run_min = state[0] if run_min is None else run_min
        run_max = state[1] if run_max is None else run_max
    if run_min.numel() != C or run_max.numel() != C:
        raise ValueError(f"running state has {run_min.numel()} channels, tensor has {C}")
    y = torch.empty_like(x) if quantize else None
    scale = torch.empty(C, dtype=torch.float64, device=dev)
    zp = torch.empty(C, dtype=torch.float64, device=dev)
    mask = H.mask_buffer(C, rowlen, dev) if (want_mask and quantize) else None
    codes = (torch.empty(x.shape, dtype=torch.int8 if qmin < 0 else torch.uint8, device=dev)
             if (want_codes and quantize) else None)
    rstats = torch.empty(C, 3, dtype=torch.float64, device=dev) if want_row_stats else None
    rc = H.lib().vsiq_pc_observe_fq_f32(H.ptr(x), H.ptr(y), H.ptr(codes), H.ptr(mask), _i64(C),
                                        _i64(rowlen), H.ptr(run_min), H.ptr(run_max), H.ptr(scale),
                                        H.ptr(zp), H.ptr(rstats), int(bool(symmetric)), int(qmin),
                                        int(qmax), qden(symmetric, obs_bits, eps), float(eps),
                                        H.stream_of(dev))
    H.check(rc, "vsiq_pc_observe_fq_f32")
    return dict(y=y, scale=scale, zp=zp, run_min=run_min, run_max=run_max, mask=mask, codes=codes,
                row_stats=rstats)


def torch_mean(x: torch.Tensor, act=None, ref=None) -> torch.Tensor:
    """K11: fp32[4] {sum|act(x)|, sum act(x), mean|act(x)|, mean act(x)} bit for bit as
    torch's CPU kernel sums them on a host of layout ``ref`` = (vec, threads) (default
    H.mean_reference(), else this process's threads) -- quantization_manager.py:66-67's
    torch.mean(torch.abs(x)) / torch.mean(x).  On x's device (CPU tensors: the host loop)."""
    if ref is None:
        ref = H.mean_reference() or (8, torch.get_num_threads())
    vec, threads = int(ref[0]), int(ref[1])
    from . import host
    if host.is_host(x):
        x = x.contiguous()
        out = torch.empty(4, dtype=torch.float32)
        rc = H.lib().vsiq_host_torch_mean_f32(H.ptr(x), _i64(x.numel()), H.act_code(act), vec, threads, H.ptr(out))
        H.check(rc, "vsiq_host_torch_mean_f32")
        return out
    x = H.require_device_f32(x)
    nb = int(H.lib().vsiq_torch_mean_ws_bytes(_i64(x.numel()), vec, threads))
    if nb < 0:
        raise ValueError(f"torch_mean: unsupported layout {ref} for {x.numel()} elements")
    ws = torch.empty(max(nb, 8), dtype=torch.uint8, device=x.device)
    out = torch.empty(4, dtype=torch.float32, device=x.device)
    rc = H.lib().vsiq_torch_mean_f32(H.ptr(x), _i64(x.numel()), H.act_code(act), vec, threads, H.ptr(out), None,
                                     H.ptr(ws), _i64(ws.numel()), H.stream_of(x.device))
    H.check(rc, "vsiq_torch_mean_f32")
    return out


def torch_stats(x: torch.Tensor, act=None, ref=None) -> torch.Tensor:
    """f64[3] {mean|act(x)|, mean act(x), std act(x)} as quantization_manager.py:66-68
    records them on a host of layout ``ref`` (torch.mean / torch.std of the fp32 tensor,
    .item()-ed): K11 and its std pass (vsiq_torch_mean_f32 with a stats record), on x's
    device.  CPU tensors: torch_mean's two means and NaN for std (the host observer's
    record holds the host std)."""
    from . import host
    if host.is_host(x):
        m = torch_mean(x, act=act, ref=ref)
        return torch.stack([m[2].double(), m[3].double(), torch.tensor(float("nan"), dtype=torch.float64)])
    if ref is None:
        ref = H.mean_reference() or (8, torch.get_num_threads())
    vec, threads = int(ref[0]), int(ref[1])
    x = H.require_device_f32(x)
    nb = int(H.lib().vsiq_torch_mean_ws_bytes(_i64(x.numel()), vec, threads))
    if nb < 0:
        raise ValueError(f"torch_stats: unsupported layout {ref} for {x.numel()} elements")
    ws = torch.empty(max(nb, 8), dtype=torch.uint8, device=x.device)
    st = torch.empty(H.ST_LEN, dtype=torch.float64, device=x.device)   # the three fields read are all written
    rc = H.lib().vsiq_torch_mean_f32(H.ptr(x), _i64(x.numel()), H.act_code(act), vec, threads, None, H.ptr(st),
                                     H.ptr(ws), _i64(ws.numel()), H.stream_of(x.device))
    H.check(rc, "vsiq_torch_mean_f32")
    return st[H.ST_MEANABS:H.ST_STD + 1]


def stats_from_row_sums(row_stats: torch.Tensor, numel: int) -> torch.Tensor:
    """[C,3] per-row (sum|x|, sum x, sum x^2) -> f64[3] fp32-rounded (mean|x|, mean, std)
    (quantization_manager.py:66-68), on the device, no sync."""
    tot = row_stats.sum(0)
    n = float(numel)
    mean = tot[1] / n
    var = (tot[2] - tot[1] * mean) / (n - 1.0) if numel > 1 else torch.full_like(mean, float("nan"))
    out = torch.stack([tot[0] / n, mean, var.clamp_min(0.0).sqrt()])
    return out.to(torch.float32).to(torch.float64)


def _pc_view(x: torch.Tensor, axis: int):
    """(rows, rowlen, channels) of the row view of x for per-channel axis 0 or 1."""
    if axis not in (0, 1) or x.dim() <= axis:
        raise ValueError(f"per-channel axis must be 0 or 1 of a tensor with more dims, got {axis}")
    C = x.shape[axis]
    rows = C if axis == 0 else x.shape[0] * C
    if rows == 0:
        return 0, 1, max(C, 1)
    return rows, x.numel() // rows, C


def _per_channel_f64(v, C, dev, what):
    t = v.detach().to(dev, torch.float64).reshape(-1).contiguous()
    if t.numel() == 1 and C > 1:
        t = t.expand(C).contiguous()
    if t.numel() != C:
        raise RuntimeError(f"per-channel {what} has {t.numel()} entries, the tensor has {C} channels")
    return t


def per_channel_fake_quant(x, scale: torch.Tensor, zp, qmin, qmax, *, zp_round=False,
                           want_mask=False, want_codes=False, axis=0):
    """Per-channel fake quant with given [C] qparams (any float dtype; zp may be None = 0)
    along ``axis`` 0 ([C, ...] weights) or 1 ([N, C, ...] activations)."""
    x = H.require_device_f32(x)
    dev = x.device
    rows, rowlen, C = _pc_view(x, axis)
    y = torch.empty_like(x)
    mask = H.mask_buffer(rows, rowlen, dev) if want_mask else None
    codes = (torch.empty(x.shape, dtype=torch.int8 if qmin < 0 else torch.uint8, device=dev)
             if want_codes else None)
    s = _per_channel_f64(scale, C, dev, "scale")
    z = _per_channel_f64(zp, C, dev, "zero point") if zp is not None else None
    rc = H.lib().vsiq_pcm_fq_fwd_f32(H.ptr(x), H.ptr(y), H.ptr(codes), H.ptr(mask), _i64(rows),
                                     _i64(rowlen), _i64(C), H.ptr(s), H.ptr(z), int(bool(zp_round)),
                                     int(qmin), int(qmax), H.stream_of(dev))
    H.check(rc, "vsiq_pcm_fq_fwd_f32")
    return y, mask, codes


class PerChannelFQFn(torch.autograd.Function):
    """Per-channel fake quant with given [C] qparams and the STE backward."""

    @staticmethod
    def forward(ctx, x, scale, zp, qmin, qmax, axis=0):
        y, mask, _ = per_channel_fake_quant(x, scale, zp, qmin, qmax, want_mask=True, axis=axis)
        rows, rowlen, C = _pc_view(x, axis)
        s = _per_channel_f64(scale, C, x.device, "scale")
        if rows != C:   # axis 1: the STE kernel takes one scale per row
            s = s.repeat(rows // C)
        ctx.save_for_backward(mask, s)
        ctx.rowlen = rowlen
        return y

    @staticmethod
    def backward(ctx, gy):
        mask, scale = ctx.saved_tensors
        return ste_backward(gy.contiguous(), mask, scale, ctx.rowlen), None, None, None, None, None


def pc_lsq_backward(g, x, scale, zp, qmin, qmax, gscale, learn_zp, axis):
    """K6: (grad_x, grad_scale f64 [C], grad_zp f64 [C])."""
    g = H.require_device_f32(g, "grad_output")
    dev = g.device
    rows, rowlen, C = _pc_view(x, axis)
    s = _per_channel_f64(scale, C, dev, "scale")
    z = _per_channel_f64(zp, C, dev, "zero point") if zp is not None else None
    gx = torch.empty_like(g)
    gs = torch.empty(C, dtype=torch.float64, device=dev)
    gz = torch.empty(C, dtype=torch.float64, device=dev)
    ws = torch.empty(max(1, int(H.lib().vsiq_pcm_workspace_doubles(rows, rowlen))), dtype=torch.float64,
                     device=dev)
    cnt = H.workspace(dev).channel_counters(C)   # per (device, stream / capture): the fold in the launch
    rc = H.lib().vsiq_pcm_lsq_bwd_arrive_f32(H.ptr(g), H.ptr(x), H.ptr(gx), _i64(rows), _i64(rowlen), _i64(C),
                                             H.ptr(s), H.ptr(z), int(bool(learn_zp)), int(qmin), int(qmax),
                                             float(gscale), H.ptr(gs), H.ptr(gz), H.ptr(ws), _i64(ws.numel()),
                                             H.ptr(cnt), _i64(cnt.numel()), H.stream_of(dev))
    H.check(rc, "vsiq_pcm_lsq_bwd_arrive_f32")
    return gx, gs, gz


class PerChannelLearnFn(torch.autograd.Function):
    """Learnable per-channel fake quant (K3-fixed forward, K6 backward): LSQFakeQuantize's
    per-channel path (quantizers/lsq_module.py:134-166) and the learnable
    PerChannelUniformQuantizer.  scale / zero_point are [C]-element tensors (any shape
    with C elements, any float dtype); their gradients come back in that shape/dtype,
    already multiplied by ``gscale`` (ScaleGradient, uniform.py:242-255)."""

    @staticmethod
    def forward(ctx, x, scale, zero_point, qmin, qmax, gscale, learn_zp, axis):
        x = H.require_device_f32(x)
        y, _, _ = per_channel_fake_quant(x, scale, zero_point, qmin, qmax, zp_round=learn_zp, axis=axis)
        ctx.save_for_backward(x)
        ctx.scale, ctx.zp = scale, zero_point
        ctx.args = (qmin, qmax, gscale, learn_zp, axis)
        return y

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        qmin, qmax, gscale, learn_zp, axis = ctx.args
        s, z = ctx.scale, ctx.zp
        gx, gs, gz = pc_lsq_backward(gy.contiguous(), x, s, z, qmin, qmax, gscale, learn_zp, axis)
        out_s = out_z = None
        if isinstance(s, torch.Tensor) and ctx.needs_input_grad[1]:
            out_s = gs.to(device=s.device, dtype=s.dtype).reshape(s.shape)
        if learn_zp and isinstance(z, torch.Tensor) and ctx.needs_input_grad[2]:
            out_z = gz.to(device=z.device, dtype=z.dtype).reshape(z.shape)
        return gx, out_s, out_z, None, None, None, None, None


class PerChannelObserveFQFn(torch.autograd.Function):
    """Per-channel observe + fake quant with the STE backward (row c uses fp32(scale_c))."""

    @staticmethod
    def forward(ctx, x, symmetric, qmin, qmax, obs_bits, eps, run_min, run_max, want_row_stats):
        r = per_channel_observe_fq(x, symmetric=symmetric, qmin=qmin, qmax=qmax, obs_bits=obs_bits,
                                   eps=eps, run_min=run_min, run_max=run_max, want_mask=True,
                                   want_row_stats=want_row_stats)
        ctx.save_for_backward(r["mask"], r["scale"])
        ctx.rowlen = x.numel() // x.shape[0]
        rs = r["row_stats"] if want_row_stats else r["scale"].new_zeros(0)
        ctx.mark_non_differentiable(r["scale"], r["zp"], rs)
        return r["y"], r["scale"], r["zp"], rs

    @staticmethod
    def backward(ctx, gy, _gs, _gz, _gr):
        mask, scale = ctx.saved_tensors
        gx = ste_backward(gy.contiguous(), mask, scale, ctx.rowlen)
        return gx, None, None, None, None, None, None, None, None
