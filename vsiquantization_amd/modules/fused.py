"""Fused QAT layers (reference: modules/fused.py:32-412).

Same class names, positional constructor signatures and attributes
(``conv_fuse``/``linear_fuse``, ``is_fuse_bn``, ``is_relu``, ``bn`` when not
folded, plus FakeQuantize's ``weight_quantizer``/``activation_quantizer``), so
``fuse_modules_unified`` builds them unchanged.  Conv / linear stay on
MIOpen / hipBLASLt through ``F.conv2d`` / ``F.linear`` (dense contractions are out
of scope); the weight and activation fake-quant go through the HIP kernels via
the managers.

BatchNorm folding happens once at construction (fused.py:100-108, 294-300):
    W' = W * (gamma / sqrt(var + eps))      b' = beta + (b - mean) * gamma / sqrt(var + eps)
Divergence from the reference (documented): Linear*/Linear with a bias no
longer evaluate ``bool(tensor)`` (fused.py:367,402 raise for out_features > 1)
and LinearBn* accept a bias-free Linear (fused.py:281 dereferences it).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..fakequant import activation
from ..quantizers.fake_quantize import FakeQuantize


def _clone_conv(cv: nn.Conv2d, with_bias: bool) -> nn.Conv2d:
    return nn.Conv2d(cv.in_channels, cv.out_channels, kernel_size=cv.kernel_size, stride=cv.stride,
                     padding=cv.padding, dilation=cv.dilation, groups=cv.groups, bias=with_bias)


def _bn_fold(weight, bias, bn, view):
    """(W * gamma/std, beta + (b - mean) * gamma/std) with std = sqrt(running_var + eps).

    On a GPU module this is one HIP launch (vsiq_bn_fold_f32); a module still on the host
    (the usual fuse-then-.cuda() flow) folds with the same torch ops as the reference."""
    if weight.device.type == "cuda" and weight.dtype == torch.float32:
        return bn_fold_device(weight, bias, bn)
    gamma = bn.weight.data.clone()
    beta = bn.bias.data.clone()
    std = torch.sqrt(bn.running_var.data.clone() + bn.eps)
    w = weight * (gamma / std).reshape(view)
    b = beta + (bias - bn.running_mean.data.clone()) * (gamma / std)
    return w, b


def bn_fold_device(weight, bias, bn):
    """BatchNorm fold on the device (k_bnfold.hip), bit-identical to the torch ops above."""
    from .. import _hip as H
    dev = weight.device
    w = weight.detach().contiguous()
    rows = w.shape[0]
    f32 = lambda t: t.detach().to(dev, torch.float32).contiguous()   # noqa: E731
    b = f32(bias) if isinstance(bias, torch.Tensor) else None
    w_out = torch.empty_like(w)
    b_out = torch.empty(rows, dtype=torch.float32, device=dev)
    rc = H.lib().vsiq_bn_fold_f32(H.ptr(w), H.ptr(b), H.ptr(f32(bn.weight)), H.ptr(f32(bn.bias)),
                                  H.ptr(f32(bn.running_mean)), H.ptr(f32(bn.running_var)), float(bn.eps),
                                  H.ptr(w_out), H.ptr(b_out), H.c_i64(rows), H.c_i64(w.numel() // max(rows, 1)),
                                  H.stream_of(dev))
    H.check(rc, "vsiq_bn_fold_f32")
    return w_out, b_out


def _activation(x, is_relu):
    return activation(x, "relu" if is_relu else "silu")   # SiLU: HIP, torch CPU's bits


class _FusedActCore(FakeQuantize):
    """Shared forward of the fused layers.

    ``run_forward_core`` keeps the reference's conv/linear -> (BN) -> ReLU/SiLU.
    When the output is quantized, ``forward`` instead hands the pre-activation to
    the activation quantizer with ``act=`` (K5): ReLU/SiLU, the activation
    observer and the fake quant then run on the conv output in one pass, and the
    backward returns the gradient with respect to the pre-activation directly."""

    has_act = True

    def _pre_act(self, x, weights, bias):
        raise NotImplementedError

    def run_forward_core(self, x, weights, bias):
        x = self._pre_act(x, weights, bias)
        return _activation(x, self.is_relu) if self.has_act else x

    def forward(self, x):
        if not (self.has_act and self.quantize_out):
            return super().forward(x)
        if self.quantize_inp:
            x = self.quantize_activation(x)
        w, b = self.get_weight_bias()
        c = self._pre_act(x, self.quantize_weights(w), b)
        return self.activation_quantizer.quantize(c, act="relu" if self.is_relu else "silu")


class _ConvCore(_FusedActCore):
    """conv2d (+ unfolded BN) (+ ReLU/SiLU) core shared by the Conv* layers."""

    def _pre_act(self, x, weights, bias):
        c = self.conv_fuse
        x = F.conv2d(x, weights, bias, stride=c.stride, padding=c.padding, dilation=c.dilation,
                     groups=c.groups)
        if not getattr(self, "is_fuse_bn", True):
            x = self.bn(x)
        return x


class ConvBnReLU(_ConvCore):
    def __init__(self, cv, bn, relu, observer_w_name: str, quantizer_w_name: str,
                 observer_a_name: str, quantizer_a_name: str, w_symmetric: bool = True,
                 a_symmetric: bool = True, is_fuse_bn=True, bits_w: int = 8, bits_a: int = 8):
        super().__init__(observer_w_name, quantizer_w_name, observer_a_name, quantizer_a_name,
                         w_symmetric, a_symmetric, bits_w, bits_a)
        self.conv_fuse = _clone_conv(cv, bool(is_fuse_bn) or cv.bias is not None)
        self.is_fuse_bn = is_fuse_bn
        self.is_relu = isinstance(relu, nn.ReLU)   # otherwise SiLU
        w = cv.weight.data.clone()
        b = cv.bias.data.clone() if cv.bias is not None else 0
        if is_fuse_bn:
            w, b = _bn_fold(w, b, bn, [-1, 1, 1, 1])
        else:
            self.bn = bn
        self.conv_fuse.weight.data.copy_(w)
        if self.conv_fuse.bias is not None:
            self.conv_fuse.bias.data.copy_(b)


class ConvBn(ConvBnReLU):
    has_act = False

    def __init__(self, cv, bn, observer_w_name: str, quantizer_w_name: str, observer_a_name: str,
                 quantizer_a_name: str, w_symmetric: bool = True, a_symmetric: bool = True,
                 is_fuse_bn=True, bits_w: int = 8, bits_a: int = 8):
        super().__init__(cv, bn, None, observer_w_name, quantizer_w_name, observer_a_name,
                         quantizer_a_name, w_symmetric, a_symmetric, is_fuse_bn, bits_w, bits_a)


class ConvReLU(_ConvCore):
    def __init__(self, cv, relu, observer_w_name: str, quantizer_w_name: str, observer_a_name: str,
                 quantizer_a_name: str, w_symmetric: bool = True, a_symmetric: bool = True,
                 bits_w: int = 8, bits_a: int = 8):
        super().__init__(observer_w_name, quantizer_w_name, observer_a_name, quantizer_a_name,
                         w_symmetric, a_symmetric, bits_w, bits_a)
        self.conv_fuse = _clone_conv(cv, cv.bias is not None)
        self.conv_fuse.weight.data.copy_(cv.weight.data)
        if cv.bias is not None:
            self.conv_fuse.bias.data.copy_(cv.bias.data)
        self.is_relu = isinstance(relu, nn.ReLU)


class Conv(_ConvCore):
    has_act = False

    def __init__(self, cv, observer_w_name: str, quantizer_w_name: str, observer_a_name: str,
                 quantizer_a_name: str, w_symmetric: bool = True, a_symmetric: bool = True,
                 bits_w: int = 8, bits_a: int = 8):
        super().__init__(observer_w_name, quantizer_w_name, observer_a_name, quantizer_a_name,
                         w_symmetric, a_symmetric, bits_w, bits_a)
        self.conv_fuse = _clone_conv(cv, cv.bias is not None)
        self.conv_fuse.weight.data.copy_(cv.weight.data)
        if cv.bias is not None:
            self.conv_fuse.bias.data.copy_(cv.bias.data)


class _LinearCore(_FusedActCore):
    def get_weight_bias(self):
        return self.linear_fuse.weight, self.linear_fuse.bias

    def _pre_act(self, x, weights, bias):
        x = F.linear(x, weights, bias)
        if not getattr(self, "is_fuse_bn", True):
            x = self.bn(x)
        return x

    def _copy_linear(self, linear):
        self.linear_fuse = nn.Linear(linear.in_features, linear.out_features,
                                     bias=linear.bias is not None)
        self.linear_fuse.weight.data.copy_(linear.weight.data)
        if linear.bias is not None:
            self.linear_fuse.bias.data.copy_(linear.bias.data)


class LinearBnReLU(_LinearCore):
    def __init__(self, linear, bn, relu, observer_w_name: str, quantizer_w_name: str,
                 observer_a_name: str, quantizer_a_name: str, w_symmetric: bool = True,
                 a_symmetric: bool = True, is_fuse_bn: bool = True, bits_w: int = 8, bits_a: int = 8):
        super().__init__(observer_w_name, quantizer_w_name, observer_a_name, quantizer_a_name,
                         w_symmetric, a_symmetric, bits_w, bits_a)
        self.linear_fuse = nn.Linear(linear.in_features, linear.out_features,
                                     bias=bool(is_fuse_bn) or linear.bias is not None)
        self.is_fuse_bn = is_fuse_bn
        self.is_relu = isinstance(relu, nn.ReLU)
        w = linear.weight.data.clone()
        b = linear.bias.data.clone() if linear.bias is not None else 0
        if is_fuse_bn:
            w, b = _bn_fold(w, b, bn, [-1, 1])
        else:
            self.bn = bn
        self.linear_fuse.weight.data.copy_(w)
        if self.linear_fuse.bias is not None:
            self.linear_fuse.bias.data.copy_(b)


class LinearBn(LinearBnReLU):
    has_act = False

    def __init__(self, linear, bn, observer_w_name: str, quantizer_w_name: str,
                 observer_a_name: str, quantizer_a_name: str, w_symmetric: bool = True,
                 a_symmetric: bool = True, is_fuse_bn: bool = True, bits_w: int = 8, bits_a: int = 8):
        super().__init__(linear, bn, None, observer_w_name, quantizer_w_name, observer_a_name,
                         quantizer_a_name, w_symmetric, a_symmetric, is_fuse_bn, bits_w, bits_a)


class LinearReLU(_LinearCore):
    def __init__(self, linear, relu, observer_w_name: str, quantizer_w_name: str,
                 observer_a_name: str, quantizer_a_name: str, w_symmetric: bool = True,
                 a_symmetric: bool = True, bits_w: int = 8, bits_a: int = 8):
        super().__init__(observer_w_name, quantizer_w_name, observer_a_name, quantizer_a_name,
                         w_symmetric, a_symmetric, bits_w, bits_a)
        self._copy_linear(linear)
        self.is_relu = isinstance(relu, nn.ReLU)


class Linear(_LinearCore):
    has_act = False

    def __init__(self, linear, observer_w_name: str, quantizer_w_name: str, observer_a_name: str,
                 quantizer_a_name: str, w_symmetric: bool = True, a_symmetric: bool = True,
                 bits_w: int = 8, bits_a: int = 8):
        super().__init__(observer_w_name, quantizer_w_name, observer_a_name, quantizer_a_name,
                         w_symmetric, a_symmetric, bits_w, bits_a)
        self._copy_linear(linear)


FUSED_CLASSES = (ConvBnReLU, ConvBn, ConvReLU, Conv, LinearBnReLU, LinearBn, LinearReLU, Linear)
