"""LSQFakeQuantize on MI355X (reference: quantizers/lsq_module.py:73-396).

A ``torch.ao.quantization.FakeQuantize`` subclass with the reference's constructor
``(learn_scale=False, config_act=False, observer=MovingAverageMinMaxObserver,
quant_min=None, quant_max=None, **observer_kwargs)``, flags (``learn_scale``,
``config_act``, ``flag_param_quant``, ``flag_adaptive``), learnable fp32
``scale_param`` / ``zero_point_param_float`` registered on the first observed
batch (and ``theta`` / ``gamma`` for weights), and ``forward`` flow:

  observer enabled   torch.ao observer -> scale / zero_point buffers (-> params)
  fake quant enabled learnable: ScaleGradient(scale_param, grad_scale) and
                     ScaleGradient(clamp(round(zero_point_param_float))), grad_scale =
                     (quant_max * numel[/C]) ** -0.5 (x 5000 for activations,
                     lsq_module.py:148-152); else the scale / zero_point buffers.

The fake quant itself runs in the HIP kernels: per-tensor K1 forward + K4 backward,
per-channel (the reference broadcasts the parameters along dim 1,
lsq_module.py:141-143) K3-fixed forward + K6 backward -- bit-exact fp32 forward and
grad_x, f64-summed parameter gradients.  CPU tensors take the native host loops
(host.py: per tensor vsiq_host_*, per channel vsiq_host_pcm_* over the [N, C, ...]
rows), with the same bits.  The observer (torch.ao, third-party) and the experimental
adaptive rounding (``flag_adaptive``, theta/gamma; the reference never sets it,
lsq_module.py:93) keep the reference's torch implementation.
"""
from __future__ import annotations

import torch
from torch.ao.quantization import FakeQuantize, MovingAverageMinMaxObserver

from .. import host as _host
from ..fakequant import PerChannelFQFn, PerChannelLearnFn, fake_quant_fixed, fake_quant_learn


class ScaleGradient(torch.autograd.Function):
    """Identity forward, gradient x scale (lsq_module.py:449-462)."""

    @staticmethod
    def forward(ctx, x, scale):
        ctx.scale = scale
        return x

    @staticmethod
    def backward(ctx, output_grad):
        return output_grad * ctx.scale, None


class RoundStraightThrough(torch.autograd.Function):
    """round() forward, identity backward (lsq_module.py:465-479)."""

    @staticmethod
    def forward(ctx, x):
        return torch.round(x)

    @staticmethod
    def backward(ctx, output_grad):
        return output_grad


class SignSTE(torch.autograd.Function):
    """sign() forward, identity backward (lsq_module.py:427-441)."""

    @staticmethod
    def forward(ctx, x):
        return torch.sign(x)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output


class LSQFakeQuantize(FakeQuantize):
    def __init__(self, learn_scale=False, config_act=False, observer=MovingAverageMinMaxObserver,
                 quant_min=None, quant_max=None, **observer_kwargs):
        super().__init__(observer, quant_min, quant_max, **observer_kwargs)
        self.learn_scale = learn_scale
        self.flag_param_quant = False
        self.flag_adaptive = False
        self.config_act = config_act

    # ------------------------------------------------------------------ forward
    def forward(self, X):
        if self.observer_enabled[0] == 1:
            self.activation_post_process(X.detach())
            _scale, _zero_point = self.calculate_qparams()
            _scale, _zero_point = _scale.to(self.scale.device), _zero_point.to(self.zero_point.device)
            if self.scale.shape != _scale.shape:
                self.scale.resize_(_scale.shape)
                self.zero_point.resize_(_zero_point.shape)
            self.scale.copy_(_scale)
            self.zero_point.copy_(_zero_point)
            if self.learn_scale:
                scale_init = _scale
                zero_point_init = _zero_point.float()
                if self.is_per_channel:
                    view = [1] + [-1] + [1] * (len(X.shape) - 2)
                    scale_init = scale_init.view(view)
                    zero_point_init = zero_point_init.view(view)
                if not self.flag_param_quant:
                    self.register_parameter("scale_param", torch.nn.Parameter(scale_init))
                    self.register_parameter("zero_point_param_float", torch.nn.Parameter(zero_point_init))
                    if not self.config_act:
                        self.register_parameter("theta", torch.nn.Parameter(torch.ones_like(X)))
                        self.register_parameter("gamma", torch.nn.Parameter(torch.zeros_like(X)))
                        self.theta.requires_grad = False
                        self.gamma.requires_grad = False
                    self.flag_param_quant = True
                else:
                    self.scale_param.data.copy_(scale_init)
                    self.zero_point_param_float.data.copy_(zero_point_init)

        if self.fake_quant_enabled[0] == 1:
            qmin = self.activation_post_process.quant_min
            qmax = self.activation_post_process.quant_max
            if self.learn_scale and self.observer_enabled[0] == 0:
                grad_scale = self.calculate_grad_scale(X)
                if self.config_act:
                    grad_scale *= 5000
                if self.flag_adaptive:
                    return self._adaptive_reference(X, grad_scale, qmin, qmax)
                return self._learnable(X, grad_scale, qmin, qmax)
            scale, zero_point = self.scale, self.zero_point
            if self.flag_adaptive:
                if self.is_per_channel:
                    view = [1] + [-1] + [1] * (len(X.shape) - 2)
                    scale, zero_point = scale.view(view), zero_point.view(view)
                return self._fq_reference(X, scale, zero_point, qmin, qmax)
            if self.is_per_channel:
                self._check_channels(X, scale)
                if X.device.type == "cpu":   # the host loops, [N, C, ...] rows
                    if X.requires_grad and torch.is_grad_enabled():
                        return _host.PcFixedFn.apply(X, scale, zero_point, qmin, qmax, 1)
                    return _host.pc_fake_quant(X, scale, zero_point, qmin, qmax, axis=1)[0]
                return PerChannelFQFn.apply(X, scale, zero_point, qmin, qmax, 1)
            return fake_quant_fixed(X, scale, zero_point, qmin, qmax)
        return X

    def _check_channels(self, X, param):
        # the reference views the parameters as [1, C, 1, ...] and broadcasts along dim 1
        if X.dim() < 2 or (param.numel() != X.shape[1] and param.numel() != 1):
            raise RuntimeError(f"The size of tensor a ({X.shape[1] if X.dim() > 1 else 1}) must match the "
                               f"size of tensor b ({param.numel()}) at non-singleton dimension 1")

    def _learnable(self, X, grad_scale, qmin, qmax):
        s, z = self.scale_param, self.zero_point_param_float
        if self.is_per_channel:
            self._check_channels(X, s)
            if X.device.type == "cpu":   # the host loops, [N, C, ...] rows
                return _host.PcLearnFn.apply(X, s, z, qmin, qmax, float(grad_scale), True, 1)
            return PerChannelLearnFn.apply(X, s, z, qmin, qmax, float(grad_scale), True, 1)
        return fake_quant_learn(X, s, z, qmin, qmax, float(grad_scale), True)

    # ------------------------------------------------------------------ reference pieces
    def calculate_grad_scale(self, quant_tensor):
        """(quant_max * numel[/shape[1]]) ** -0.5 (lsq_module.py:314-333)."""
        num_elements_feature = quant_tensor.numel()
        if self.is_per_channel:
            num_elements_feature /= quant_tensor.shape[1]
        return (self.quant_max * num_elements_feature) ** -0.5

    def scale_grad_func(self):
        return ScaleGradient.apply

    def discretizer(self):
        return RoundStraightThrough.apply

    def signSTE(self):
        return SignSTE.apply

    def zero_point_rounding(self):
        zero_point = self.discretizer()(self.zero_point_param_float)
        return torch.clamp(zero_point, self.quant_min, self.quant_max)

    def discreate_tensor(self, x, scale, zero_point, quant_min, quant_max):
        return torch.clamp(self.discretizer()(x / scale + zero_point), quant_min, quant_max)

    def discreate_adaptive_tensor(self, x, scale, zero_point, quant_min, quant_max):
        """Adaptive rounding with theta (lsq_module.py:268-291), torch reference path."""
        x.requires_grad = False
        h_theta = torch.clamp(torch.tanh(self.theta) * 1.2, -1, 1)
        self.saved_h_theta = h_theta
        return torch.clamp(self.discretizer()(x / scale + zero_point) + h_theta, quant_min, quant_max)

    def _fq_reference(self, x, scale, zero_point, quant_min, quant_max):
        x_int = (self.discreate_adaptive_tensor if self.flag_adaptive else self.discreate_tensor)(
            x, scale, zero_point, quant_min, quant_max)
        return scale * (x_int - zero_point)

    def _adaptive_reference(self, X, grad_scale, qmin, qmax):
        scale = self.scale_grad_func()(self.scale_param, grad_scale)
        zero_point = self.scale_grad_func()(self.zero_point_rounding(), grad_scale)
        return self._fq_reference(X, scale, zero_point, qmin, qmax)

    fake_quantize_per_tensor_affine = _fq_reference
    fake_quantize_per_channel_affine = (
        lambda self, x, scale, zero_point, ch_axis, quant_min, quant_max:
        self._fq_reference(x, scale, zero_point, quant_min, quant_max))

    def fake_quantize_per_tensor_power_of_two(self, x):
        p = self.discretizer()(torch.log2(torch.abs(x)))
        return self.signSTE()(x) * torch.pow(2, p)

    def scale_weight_grad(self, quant_tensor, alpha=1):
        q = quant_tensor.clone().detach()
        s = self.scale_param.clone().detach()
        return torch.exp(-alpha * torch.abs(torch.round(q / s) - q / s))

    def scale_grad_(self, x, gamma):
        left_expr = ((0.5 - gamma) / gamma) * (x + 0.5)
        right_expr = ((0.5 - gamma) / gamma) * (x - 0.5)
        return torch.where((x >= -0.5 - gamma) & (x <= -0.5 + gamma), left_expr,
                           torch.where((x > -0.5 + gamma) & (x <= 0.5 - gamma), -x,
                                       torch.where((x > 0.5 - gamma) & (x <= 0.5 + gamma), right_expr,
                                                   torch.full_like(x, float("nan")))))

    def scale_grad_scale_param(self, quant_tensor):
        q = quant_tensor.clone().detach()
        s = self.scale_param.clone().detach()
        sub_round = torch.round(q / s) - q / s
        return torch.clamp(-self.scale_grad_(sub_round, gamma=0.1) / (sub_round + 1e-30), -2, 2)

    def activate_grad_theta(self):
        self.theta.requires_grad = True
        self.gamma.requires_grad = True
