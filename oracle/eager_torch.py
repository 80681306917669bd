"""The reference's eager-PyTorch op sequence, restated (TEST INFRASTRUCTURE / CPU BASELINE).

Used only by bench.py's ``cpu_baseline`` leg and by tests: it is what the
reference costs on the host, op for op:
  observers/minmax.py:42-47       x.min().item(), x.max().item()
  observers/minmax.py:49-74       Python float64 qparams
  quantizers/uniform.py:95        clamp(RoundSTE(x / s + zp), qmin, qmax)
  quantizers/uniform.py:55        (x_int - zp) * s
  quantizers/uniform.py:258-271   round with a straight-through gradient
"""
import torch

from .fakequant_np import minmax_qparams, qrange


class _RoundSTE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return torch.round(x)

    @staticmethod
    def backward(ctx, g):
        return g


def observe(x, min_val=0, max_val=0):
    mn = x.min().item()
    mx = x.max().item()
    if mn < min_val:
        min_val = mn
    if mx > max_val:
        max_val = mx
    return min_val, max_val


def fake_quant(x, scale, zero_point, qmin, qmax):
    x_int = torch.clamp(_RoundSTE.apply(x / scale + zero_point), qmin, qmax)
    return (x_int - zero_point) * scale


def per_channel_step(w, g, symmetric=False, bits=8):
    """Per-channel observe + fake-quant forward, then STE backward (reference classes looped)."""
    qmin, qmax = qrange(bits, symmetric)
    w = w.detach().requires_grad_(True)
    ys = []
    # unbind (not w[c]): its backward stacks the row gradients once, where 1024 SelectBackward
    # nodes would each scatter into a full-size zero gradient (quadratic in the channel count)
    for row in w.unbind(0):
        mn, mx = observe(row.detach())
        s, z = minmax_qparams(mn, mx, symmetric, 8)
        ys.append(fake_quant(row, s, z, qmin, qmax))
    torch.stack(ys).backward(g)
    return w.grad


def lsq_step(x, g, scale=0.03, bits=8, act=None, zero_point=None):
    """Learnable fake-quant fwd + bwd (uniform.py:47-56 with ScaleGradient); symmetric, or
    with ``zero_point`` (a float) the asymmetric LSQQuantizer variant: a learnable f64 zero
    point through zero_point_rounding (uniform.py:98-102, round STE + clamp) and its own
    ScaleGradient (:51-52).  act="relu"/"silu": the fused layers' activation first
    (modules/fused.py:133).  Returns (grad_x, grad_scale) (+ grad_zp when asymmetric)."""
    asym = zero_point is not None
    qmin, qmax = qrange(bits, not asym)
    s = torch.nn.Parameter(torch.tensor(scale, dtype=torch.float64))
    gscale = (qmax * x.numel()) ** -0.5
    x0 = x.detach().requires_grad_(True)
    x = x0
    if act == "relu":
        x = torch.nn.functional.relu(x0)
    elif act == "silu":
        x = torch.nn.functional.silu(x0)

    class _ScaleGrad(torch.autograd.Function):
        @staticmethod
        def forward(ctx, v):
            return v

        @staticmethod
        def backward(ctx, gv):
            return gv * gscale

    if not asym:
        y = fake_quant(x, _ScaleGrad.apply(s), 0, qmin, qmax)
        y.backward(g)
        return x0.grad, s.grad
    z = torch.nn.Parameter(torch.tensor(zero_point, dtype=torch.float64))
    zr = _ScaleGrad.apply(torch.clamp(_RoundSTE.apply(z), qmin, qmax))
    y = fake_quant(x, _ScaleGrad.apply(s), zr, qmin, qmax)
    y.backward(g)
    return x0.grad, s.grad, z.grad
