"""The fake-quant path for CPU tensors: native host loops in the same library
(csrc/k_host.hip, vsiq_host_* in include/vsiq.h) -- the reference's own environment
(BASELINE C1: UniformQuantizer / MinMaxObserver on CPU tensors).  The elementwise
outputs (y, integer codes, masks, grad_x), min / max and the f64 qparams are the HIP
kernels' bit for bit (IEEE fp32 division, rint, NaN-propagating clamp, f64 qparams,
torch CPU's SiLU).  The f64 sums (mean|x|, mean, std, scale / zero-point gradients) are
summed in 16 lanes per 64K chunk, folded in lane then chunk order -- the same bits with
or without AVX-512 (VSIQ_HOST_SIMD=0) and for any thread count, but a different order
from the GPU's tree (equal to it within the f64 rounding of the sum).  This is not a
fallback for CUDA tensors: a CUDA tensor never comes here, and a missing library raises
like every other op.
"""
from __future__ import annotations

import numbers

import numpy as np
import torch

from . import _hip as H


def is_host(x) -> bool:
    """A CPU float32 tensor (the host path's input)."""
    return isinstance(x, torch.Tensor) and x.device.type == "cpu" and x.dtype == torch.float32


def _i64(n):
    return H.c_i64(int(n))


def _num(v) -> float:
    if isinstance(v, torch.Tensor):
        if v.numel() != 1:
            raise ValueError(f"expected a scalar qparam, got shape {tuple(v.shape)}")
        return float(v.detach().reshape(()).item())
    if isinstance(v, (numbers.Real, np.floating, np.integer)):
        return float(v)
    raise TypeError(f"unsupported qparam type {type(v).__name__}")


def _f32(x, what="x"):
    if x.dtype != torch.float32:
        raise TypeError(f"{what}: only float32 is supported by the fake-quant path, got {x.dtype}")
    return x.contiguous()


def fake_quant(x, scale, zero_point, qmin, qmax, *, zp_round=False, qp=None, want_mask=False, want_codes=False,
               discrete=False, act=None):
    """Host counterpart of fakequant.fake_quant: (y, mask uint8 | None, codes | None)."""
    x = _f32(x)
    y = torch.empty_like(x)
    mask = torch.empty(x.shape, dtype=torch.uint8) if want_mask else None
    codes = torch.empty(x.shape, dtype=torch.int8 if qmin < 0 else torch.uint8) if want_codes else None
    if qp is not None:
        qp = qp.detach().to("cpu", torch.float64).contiguous()
        s = z = 0.0
    else:
        s, z = _num(scale), _num(zero_point)
    rc = H.lib().vsiq_host_fq_fwd_f32(H.ptr(x), H.ptr(y), H.ptr(codes), H.ptr(mask), _i64(x.numel()), H.act_code(act),
                                      H.ptr(qp), s, z, int(bool(zp_round)), int(bool(discrete)), int(qmin), int(qmax))
    H.check(rc, "vsiq_host_fq_fwd_f32")
    return y, mask, codes


class FixedFn(torch.autograd.Function):
    """Fixed-qparam fake quant with the reference's STE gradient, on the host."""

    @staticmethod
    def forward(ctx, x, scale, zero_point, qmin, qmax, qp, act=None):
        y, mask, _ = fake_quant(x, scale, zero_point, qmin, qmax, qp=qp, want_mask=True, act=act)
        ctx.code = H.act_code(act)
        ctx.save_for_backward(mask, x.contiguous())
        ctx.scale = float(qp[H.QP_SCALE]) if qp is not None else _num(scale)
        return y

    @staticmethod
    def backward(ctx, gy):
        mask, x = ctx.saved_tensors
        g = _f32(gy, "grad_output")
        gx = torch.empty_like(g)
        rc = H.lib().vsiq_host_ste_bwd_f32(H.ptr(g), H.ptr(mask), H.ptr(x), H.ptr(gx), _i64(g.numel()), ctx.code,
                                           ctx.scale)
        H.check(rc, "vsiq_host_ste_bwd_f32")
        return gx, None, None, None, None, None, None


class LearnFn(torch.autograd.Function):
    """Learnable fake quant (uniform.py:47-56) on the host: forward as fake_quant with the
    (rounded, clamped) zero point, backward grad_x + the f64 closed-form scale / zero-point
    gradients times the ScaleGradient factor."""

    @staticmethod
    def forward(ctx, x, scale, zero_point, qmin, qmax, gscale, learn_zp, act=None):
        x = _f32(x)
        y, _, _ = fake_quant(x, scale, zero_point, qmin, qmax, zp_round=learn_zp == 1, act=act)
        ctx.save_for_backward(x)
        ctx.scale, ctx.zp = scale, zero_point
        ctx.args = (int(qmin), int(qmax), float(gscale), int(learn_zp), H.act_code(act))
        return y

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        qmin, qmax, gscale, learn_zp, code = ctx.args
        s, z = ctx.scale, ctx.zp
        g = _f32(gy, "grad_output")
        gx = torch.empty_like(g)
        grads = torch.empty(2, dtype=torch.float64)
        rc = H.lib().vsiq_host_lsq_bwd_f32(H.ptr(g), H.ptr(x), H.ptr(gx), _i64(g.numel()), code, _num(s), _num(z),
                                           int(learn_zp), qmin, qmax, gscale, H.ptr(grads))
        H.check(rc, "vsiq_host_lsq_bwd_f32")
        gs = gz = None
        if isinstance(s, torch.Tensor) and ctx.needs_input_grad[1]:
            gs = grads[0].to(device=s.device, dtype=s.dtype).reshape(s.shape)
        if learn_zp and isinstance(z, torch.Tensor) and ctx.needs_input_grad[2]:
            gz = grads[1].to(device=z.device, dtype=z.dtype).reshape(z.shape)
        return gx, gs, gz, None, None, None, None, None


def fake_quant_fixed(x, scale, zero_point, qmin, qmax, qp=None, act=None):
    if x.requires_grad and torch.is_grad_enabled():
        return FixedFn.apply(x, scale, zero_point, qmin, qmax, qp, act)
    return fake_quant(x, scale, zero_point, qmin, qmax, qp=qp, act=act)[0]


def fake_quant_learn(x, scale, zero_point, qmin, qmax, gscale, learn_zp, act=None):
    return LearnFn.apply(x, scale, zero_point, qmin, qmax, gscale, learn_zp, act)


def observe_tensor(x, *, symmetric, num_bits=8, eps=1e-8, run_minmax=None, want_qp=True, want_stats=True,
                   act=None):
    """Host counterpart of fakequant.observe_tensor: one pass -> running update (fp32[2]
    CPU state) -> f64 qparams record, stats record."""
    from .fakequant import qden
    x = _f32(x)
    if x.numel() == 0:
        raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0.")
    qp = torch.empty(H.QP_LEN, dtype=torch.float64) if want_qp else None
    st = torch.empty(H.ST_LEN, dtype=torch.float64) if want_stats else None
    if run_minmax is not None and (run_minmax.device.type != "cpu" or run_minmax.dtype != torch.float32):
        raise ValueError("host observe: the running state must be a CPU float32 tensor")
    rc = H.lib().vsiq_host_observe_f32(H.ptr(x), _i64(x.numel()), H.act_code(act), H.ptr(st), H.ptr(run_minmax),
                                       H.ptr(qp), int(bool(symmetric)), qden(symmetric, num_bits, eps), float(eps))
    H.check(rc, "vsiq_host_observe_f32")
    return qp, st


# --------------------------------------------------------------------------- per-channel
def _rows(x):
    C = x.shape[0] if x.dim() > 0 else 1
    if C == 0 or x.numel() == 0:
        raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0.")
    return C, x.numel() // C


def _pc_view(x, axis):
    """(rows, rowlen, channels) of per-channel ``axis`` 0 ([C, ...] weights: one row per
    channel) or 1 ([N, C, ...] activations: N * C rows, row r in channel r % C) -- the
    device path's view (fakequant._pc_view)."""
    if axis == 0:
        C, rowlen = _rows(x)
        return C, rowlen, C
    if axis != 1 or x.dim() < 2:
        raise ValueError(f"per-channel axis must be 0 or 1 of a tensor with more dims, got {axis}")
    C, rows = x.shape[1], x.shape[0] * x.shape[1]
    if rows == 0 or x.numel() == 0:
        raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0.")
    return rows, x.numel() // rows, C


def _row_f64(v, C, what):
    t = (v.detach() if isinstance(v, torch.Tensor) else torch.tensor(float(v))).to("cpu", torch.float64)
    t = t.reshape(-1)
    if t.numel() == 1 and C > 1:
        t = t.expand(C)
    if t.numel() != C:
        raise RuntimeError(f"per-channel {what} has {t.numel()} entries, the tensor has {C} channels")
    return t.contiguous()


def pc_observe_fq(x, *, symmetric, qmin, qmax, obs_bits=8, eps=1e-8, run_min=None, run_max=None,
                  quantize=True, want_mask=False, want_row_stats=False):
    """Host counterpart of fakequant.per_channel_observe_fq (K3): each out-channel row W[c]
    observed (running state per row) and fake-quantized with its own f64 qparams, the
    per-tensor host code on each row.  Same dict as the device function."""
    from .fakequant import qden
    x = _f32(x)
    C, rowlen = _rows(x)
    if run_min is None or run_max is None:
        state = torch.zeros(2, C, dtype=torch.float32)
        run_min = state[0] if run_min is None else run_min
        run_max = state[1] if run_max is None else run_max
    for r in (run_min, run_max):
        if r.numel() != C or r.device.type != "cpu" or r.dtype != torch.float32 or not r.is_contiguous():
            raise ValueError(f"host per-channel observe: running state must be contiguous CPU float32 [{C}]")
    y = torch.empty_like(x) if quantize else None
    mask = torch.empty(x.shape, dtype=torch.uint8) if (want_mask and quantize) else None
    scale = torch.empty(C, dtype=torch.float64)
    zp = torch.empty(C, dtype=torch.float64)
    rstats = torch.empty(C, 3, dtype=torch.float64) if want_row_stats else None
    rc = H.lib().vsiq_host_pc_observe_fq_f32(H.ptr(x), H.ptr(y), H.ptr(mask), _i64(C), _i64(rowlen), H.ptr(run_min),
                                             H.ptr(run_max), H.ptr(scale), H.ptr(zp), H.ptr(rstats),
                                             int(bool(symmetric)), qden(symmetric, obs_bits, eps), float(eps),
                                             int(qmin), int(qmax))
    H.check(rc, "vsiq_host_pc_observe_fq_f32")
    return dict(y=y, scale=scale, zp=zp, run_min=run_min, run_max=run_max, mask=mask, codes=None,
                row_stats=rstats)


def pc_fake_quant(x, scale, zp, qmin, qmax, *, zp_round=False, want_mask=False, axis=0):
    """Per-channel fake quant with given [C] qparams along ``axis`` 0 or 1 on the host:
    (y, mask | None)."""
    x = _f32(x)
    rows, rowlen, C = _pc_view(x, axis)
    s = _row_f64(scale, C, "scale")
    z = _row_f64(zp, C, "zero point") if zp is not None else None
    y = torch.empty_like(x)
    mask = torch.empty(x.shape, dtype=torch.uint8) if want_mask else None
    rc = H.lib().vsiq_host_pcm_fq_fwd_f32(H.ptr(x), H.ptr(y), H.ptr(mask), _i64(rows), _i64(rowlen), _i64(C),
                                          H.ptr(s), H.ptr(z), int(bool(zp_round)), int(qmin), int(qmax))
    H.check(rc, "vsiq_host_pcm_fq_fwd_f32")
    return y, mask


def pc_ste_backward(g, mask, scale, axis=0):
    g = _f32(g, "grad_output")
    rows, rowlen, C = _pc_view(g, axis)
    s = _row_f64(scale, C, "scale")
    gx = torch.empty_like(g)
    rc = H.lib().vsiq_host_pcm_ste_bwd_f32(H.ptr(g), H.ptr(mask), H.ptr(gx), _i64(rows), _i64(rowlen), _i64(C),
                                           H.ptr(s))
    H.check(rc, "vsiq_host_pcm_ste_bwd_f32")
    return gx


class PcFixedFn(torch.autograd.Function):
    """Per-channel fake quant with given [C] qparams and the STE backward, on the host
    (``axis`` 0 or 1)."""

    @staticmethod
    def forward(ctx, x, scale, zp, qmin, qmax, axis=0):
        y, mask = pc_fake_quant(x, scale, zp, qmin, qmax, want_mask=True, axis=axis)
        ctx.save_for_backward(mask, _row_f64(scale, _pc_view(x, axis)[2], "scale"))
        ctx.axis = axis
        return y

    @staticmethod
    def backward(ctx, gy):
        mask, s = ctx.saved_tensors
        return pc_ste_backward(gy, mask, s, ctx.axis), None, None, None, None, None


class PcObserveFQFn(torch.autograd.Function):
    """Per-channel observe + fake quant with the STE backward, on the host."""

    @staticmethod
    def forward(ctx, x, symmetric, qmin, qmax, obs_bits, eps, run_min, run_max, want_row_stats):
        r = pc_observe_fq(x, symmetric=symmetric, qmin=qmin, qmax=qmax, obs_bits=obs_bits, eps=eps,
                          run_min=run_min, run_max=run_max, want_mask=True, want_row_stats=want_row_stats)
        ctx.save_for_backward(r["mask"], r["scale"])
        rs = r["row_stats"] if want_row_stats else r["scale"].new_zeros(0)
        ctx.mark_non_differentiable(r["scale"], r["zp"], rs)
        return r["y"], r["scale"], r["zp"], rs

    @staticmethod
    def backward(ctx, gy, _gs, _gz, _gr):
        mask, scale = ctx.saved_tensors
        return pc_ste_backward(gy, mask, scale), None, None, None, None, None, None, None, None


class PcLearnFn(torch.autograd.Function):
    """Learnable per-channel fake quant on the host (``axis`` 0: [C, ...] weights, 1:
    [N, C, ...] activations -- LSQFakeQuantize): each row the per-tensor learnable host
    path with its channel's scale / zero point; [C] gradients (f64 sums over each channel's
    rows) times gscale."""

    @staticmethod
    def forward(ctx, x, scale, zero_point, qmin, qmax, gscale, learn_zp, axis=0):
        x = _f32(x)
        y, _ = pc_fake_quant(x, scale, zero_point, qmin, qmax, zp_round=learn_zp, axis=axis)
        ctx.save_for_backward(x)
        ctx.scale, ctx.zp = scale, zero_point
        ctx.args = (int(qmin), int(qmax), float(gscale), int(bool(learn_zp)), axis)
        return y

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        qmin, qmax, gscale, learn_zp, axis = ctx.args
        s, z = ctx.scale, ctx.zp
        g = _f32(gy, "grad_output")
        rows, rowlen, C = _pc_view(x, axis)
        sr = _row_f64(s, C, "scale")
        zr = _row_f64(z, C, "zero point") if z is not None else None
        gx = torch.empty_like(g)
        gs = torch.empty(C, dtype=torch.float64)
        gz = torch.empty(C, dtype=torch.float64)
        rc = H.lib().vsiq_host_pcm_lsq_bwd_f32(H.ptr(g), H.ptr(x), H.ptr(gx), _i64(rows), _i64(rowlen), _i64(C),
                                               H.ptr(sr), H.ptr(zr), learn_zp, qmin, qmax, gscale, H.ptr(gs),
                                               H.ptr(gz))
        H.check(rc, "vsiq_host_pcm_lsq_bwd_f32")
        out_s = out_z = None
        if isinstance(s, torch.Tensor) and ctx.needs_input_grad[1]:
            out_s = gs.to(device=s.device, dtype=s.dtype).reshape(s.shape)
        if learn_zp and isinstance(z, torch.Tensor) and ctx.needs_input_grad[2]:
            out_z = gz.to(device=z.device, dtype=z.dtype).reshape(z.shape)
        return gx, out_s, out_z, None, None, None, None, None


def threads() -> int:
    """Host threads the CPU path uses (VSIQ_HOST_THREADS, else the CPUs this process may use)."""
    return int(H.lib().vsiq_host_threads())


def simd() -> bool:
    """True when the host loops run their AVX-512 form (csrc/host_simd.cpp)."""
    return bool(H.lib().vsiq_host_simd())


__all__ = ["is_host", "fake_quant", "fake_quant_fixed", "fake_quant_learn", "observe_tensor", "pc_observe_fq",
           "pc_fake_quant", "threads", "simd"]
