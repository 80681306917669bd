"""UniformQuantizer on MI355X (reference: quantizers/uniform.py:7-102, 242-271).

Same registry name, constructor ``(num_bits=8, symmetric=True)``, attributes
(``num_bits, symmetric, qmin, qmax, calib_grad_scale``) and ``quantize``
protocol as the reference; the arithmetic runs in the HIP kernels of
``vsiquantization_amd.fakequant`` (bit-exact with the reference's CPU path):

* fixed qparams (``is_learning_scale=False``): one launch (K1), STE backward
  from a saved uint8 mask;
* learnable (``is_learning_scale=True``): forward K1 reading the f64 scale
  Parameter on the device, backward K4 (grad_x + f64 scale/zp gradients with the
  reference's ScaleGradient factor).
"""
from __future__ import annotations

import torch

from ..fakequant import fake_quant, fake_quant_fixed, fake_quant_learn
from ..utils.registry import register_class
from .base import BaseQuantizer


class ScaleGradient(torch.autograd.Function):
    """Identity forward; backward multiplies the gradient by ``scale`` (uniform.py:242-255)."""

    @staticmethod
    def forward(ctx, x, scale):
        ctx.scale = scale
        return x

    @staticmethod
    def backward(ctx, grad):
        return grad * ctx.scale, None


class RoundStraightThrough(torch.autograd.Function):
    """round() forward, identity backward (uniform.py:258-271)."""

    @staticmethod
    def forward(ctx, x):
        return torch.round(x)

    @staticmethod
    def backward(ctx, grad):
        return grad


def _calib_factor(q):
    """Effective ``calib_grad_scale`` factor.  It may be a per-channel tensor
    (utils/estimate_bn.py:136); the reference then reduces ScaleGradient's tensor-valued
    gradient onto the 0-dim scale (sum_to, uniform.py:47-53,252-253), i.e. the factor is
    the sum (here in float64; the reference's fp32 products differ by ~1e-7 relative,
    inside the 1e-4 parity gate).  Cached per tensor and in-place version, so the host
    reads a device tensor once after estimate_bn sets it, not on every forward."""
    c = q.calib_grad_scale
    if not isinstance(c, torch.Tensor):
        return float(c)
    cache = q.__dict__.get("_calib_cache")
    if cache is None or cache[0] is not c or cache[1] != c._version:
        cache = (c, c._version, float(c.detach().to(torch.float64).sum().item()))
        q.__dict__["_calib_cache"] = cache
    return cache[2]


@register_class
class UniformQuantizer(BaseQuantizer):
    #: zero point becomes a learnable tensor in QuantizationManager.make_learn_qparameter
    #: only for quantizers that set this (the reference manager never does: qm.py:50,100-103)
    learns_zero_point = False

    def __init__(self, num_bits=8, symmetric=True):
        self.num_bits = num_bits
        self.symmetric = symmetric
        if symmetric:
            self.qmin, self.qmax = -(2 ** (num_bits - 1)), 2 ** (num_bits - 1) - 1
        else:
            self.qmin, self.qmax = 0, 2 ** num_bits - 1
        self.calib_grad_scale = 1

    # ------------------------------------------------------------------ protocol
    def quantize(self, x, scale, zero_point, is_learning_scale, act=None):
        """Fake-quantize ``x`` (uniform.py:34-56): ``(clamp(round(x/s+zp)) - zp) * s``.

        ``act`` ("relu" / "silu", an MI355X extension of the protocol): quantize
        act(x) in the same pass (K5); gradients are with respect to ``x``."""
        if not is_learning_scale:
            return fake_quant_fixed(x, scale, zero_point, self.qmin, self.qmax, act=act)
        gscale, zero_point, learn_zp = self.learn_args(x, zero_point)
        return fake_quant_learn(x, scale, zero_point, self.qmin, self.qmax, gscale, learn_zp, act)

    def learn_args(self, x, zero_point):
        """(gscale, zero_point, learn_zp) of the learnable path for input x (uniform.py:47-53):
        the ScaleGradient factor, and whether the zero point is learned (rounded + clamped
        in the forward, with a gradient)."""
        gscale = self.calculate_grad_scale(x) * _calib_factor(self)
        learn_zp = not self.symmetric
        if learn_zp and not isinstance(zero_point, torch.Tensor):
            zero_point = self._int_zero_point_learnable(zero_point)
            learn_zp = isinstance(zero_point, torch.Tensor)
        if not learn_zp and isinstance(zero_point, torch.Tensor) and zero_point.requires_grad:
            # symmetric: the reference skips zero_point_rounding / ScaleGradient on zp
            # (uniform.py:50) but autograd still reaches it through x/s + zp and
            # (x_int - zp) * s: zp as given, grad = sum g*s*(mask - 1) (zp_learn 2)
            learn_zp = 2
        return gscale, zero_point, learn_zp

    def _int_zero_point_learnable(self, zero_point):
        # Reference behaviour (uniform.py:50-52 -> :100 -> :267): torch.round(<int>) raises.
        raise TypeError(
            "round(): argument 'input' must be Tensor, not int — the reference UniformQuantizer "
            "cannot learn an integer zero point (asymmetric + is_learning_scale); use LSQQuantizer")

    def calculate_grad_scale(self, quant_tensor):
        """(qmax * numel) ** -0.5 (uniform.py:58-71)."""
        return (self.qmax * quant_tensor.numel()) ** -0.5

    def scale_grad_func(self):
        return ScaleGradient.apply

    def discretizer(self):
        return RoundStraightThrough.apply

    def discreate_tensor(self, x, scale, zero_point, quant_min, quant_max):
        """Integer codes as an fp32 tensor: clamp(round(x/s+zp), qmin, qmax) (uniform.py:81-96)."""
        return fake_quant(x, scale, zero_point, quant_min, quant_max, discrete=True)[0]

    def zero_point_rounding(self, zero_point):
        """clamp(round(zp), qmin, qmax) with a straight-through gradient (uniform.py:98-102)."""
        return torch.clamp(RoundStraightThrough.apply(zero_point), self.qmin, self.qmax)

    def __repr__(self):
        return (f"{type(self).__name__}(num_bits={self.num_bits}, symmetric={self.symmetric}, "
                f"qmin={self.qmin}, qmax={self.qmax})")
