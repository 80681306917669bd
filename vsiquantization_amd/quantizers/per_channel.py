"""PerChannelUniformQuantizer — UniformQuantizer arithmetic (quantizers/uniform.py:34-56)
with one (scale, zero point) per out-channel (axis 0), build-defined.

``quantize(x, scale, zero_point, is_learning_scale)`` takes float64 [C] device
tensors (PerChannelMinMaxObserver's output); CPU tensors run the native host loops row by
row (host.pc_fake_quant / PcLearnFn).  Scalars fall back to the
per-tensor UniformQuantizer behaviour.  Learnable (``is_learning_scale``): a [C]
scale Parameter (QuantizationManager.make_learn_qparameter) trained with the
per-channel LSQ backward (K6, the kernel LSQFakeQuantize's per-channel path uses),
gradient scale (qmax * numel / C) ** -0.5 -- the per-scale element count, as
LSQFakeQuantize.calculate_grad_scale does (quantizers/lsq_module.py:326-330).
"""
from __future__ import annotations

import torch

from .. import host as _host
from ..fakequant import PerChannelFQFn, PerChannelLearnFn, per_channel_fake_quant
from ..fakequant import activation as _activation
from ..utils.registry import register_class
from .uniform import UniformQuantizer, _calib_factor




def _per_channel(v) -> bool:
    return isinstance(v, torch.Tensor) and v.dim() == 1 and v.numel() > 1


@register_class
class PerChannelUniformQuantizer(UniformQuantizer):
    axis = 0

    def quantize(self, x, scale, zero_point, is_learning_scale, act=None):
        if not (_per_channel(scale) or _per_channel(zero_point)):
            return super().quantize(x, scale, zero_point, is_learning_scale, act=act)
        if act is not None:   # per-channel activations: activation first (torch), then K3-fixed
            x = _activation(x, act)
        C = x.shape[0]
        if is_learning_scale:
            gscale = float((self.qmax * x.numel() / C) ** -0.5) * _calib_factor(self)
            learn_zp = isinstance(zero_point, torch.Tensor) and zero_point.requires_grad
            z = zero_point if isinstance(zero_point, torch.Tensor) else torch.full(
                (C,), float(zero_point), dtype=torch.float64, device=x.device)
            if _host.is_host(x):   # CPU tensor: the per-tensor host path row by row
                return _host.PcLearnFn.apply(x, scale, z, self.qmin, self.qmax, gscale, learn_zp)
            return PerChannelLearnFn.apply(x, scale, z, self.qmin, self.qmax, gscale, learn_zp, 0)
        s = scale if isinstance(scale, torch.Tensor) else torch.full((C,), float(scale), dtype=torch.float64)
        z = zero_point if isinstance(zero_point, torch.Tensor) else torch.full((C,), float(zero_point),
                                                                                dtype=torch.float64)
        if s.numel() != C or z.numel() != C:
            raise ValueError(f"per-channel qparams have {s.numel()}/{z.numel()} entries, x has {C} channels")
        if _host.is_host(x):
            if x.requires_grad and torch.is_grad_enabled():
                return _host.PcFixedFn.apply(x, s, z, self.qmin, self.qmax)
            return _host.pc_fake_quant(x, s, z, self.qmin, self.qmax)[0]
        if x.requires_grad and torch.is_grad_enabled():
            return PerChannelFQFn.apply(x, s, z, self.qmin, self.qmax, 0)
        return per_channel_fake_quant(x, s, z, self.qmin, self.qmax)[0]
