"""Multi-tensor learnable fake quant (k_multi.hip, quantizers/foreach.py) on MI355X.

Per tensor the one-launch forward / backward must equal the per-tensor path
(FakeQuantLearnFn: K1 + K4, itself pinned to the oracle and the reference goldens)
bit for bit -- y, grad_x, and the scale / zero-point gradients (same blocks, same
fold order) -- and the oracle's closed form (oracle/fakequant_np.py
lsq_forward_backward, reference quantizers/uniform.py:47-56 autograd).
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

from vsiquantization_amd import fakequant as FQ
from vsiquantization_amd.modules.fused import ConvBnReLU
from vsiquantization_amd.quantizers.foreach import enable_multi_tensor_weights, quantize_weights_multi
from vsiquantization_amd.utils.quantize_manager import activate_learning_qparam, activate_quantizer
from oracle import fakequant_np as O
from tests import goldens as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

# YOLOv8n weight sizes, ragged sizes, one above the flat-arrival limit (2^19 + 4:
# single-tensor kernel inside the same call)
SIZES = [432, 4608, 1024, 2304, 1536, 18432, 294912, 7, 1023, 5, 2 ** 19 + 4, 131072]


def _case(n, i, asym):
    g = torch.Generator(device=DEV).manual_seed(100 + i)
    x = torch.randn(n, device=DEV, generator=g) * 0.05
    gy = torch.randn(n, device=DEV, generator=g)
    bits = (2, 4, 8)[i % 3]
    if asym:
        qmin, qmax = 0, 2 ** bits - 1
        zp = nn.Parameter(torch.tensor(float(2 ** (bits - 1)) + 0.3, dtype=torch.float64, device=DEV))
    else:
        qmin, qmax = -(2 ** (bits - 1)), 2 ** (bits - 1) - 1
        zp = 0
    s = nn.Parameter(torch.tensor(0.02 + 0.003 * i, dtype=torch.float64, device=DEV))
    gscale = (qmax * n) ** -0.5
    return x, gy, s, zp, qmin, qmax, gscale


@pytest.mark.parametrize("asym", [False, True])
@pytest.mark.parametrize("count", [len(SIZES), 40])
def test_multi_equals_per_tensor(asym, count):
    sizes = (SIZES * 3)[:count]
    cases = [_case(n, i, asym) for i, n in enumerate(sizes)]
    # multi-tensor
    xs = [c[0].clone().requires_grad_(True) for c in cases]
    specs = []
    for x, c in zip(xs, cases):
        _, _, s, zp, qmin, qmax, gscale = c
        specs.append(FQ.LsqSpec(s, zp, qmin, qmax, gscale, asym))
    ys = FQ.lsq_fake_quant_multi(xs, specs)
    torch.autograd.backward(ys, [c[1] for c in cases])
    got = [(y.detach().clone(), x.grad.clone(), c[2].grad.clone(),
            c[3].grad.clone() if asym else None) for x, y, c in zip(xs, ys, cases)]
    for c in cases:
        c[2].grad = None
        if asym:
            c[3].grad = None
    # per tensor (FakeQuantLearnFn)
    for (x0, gy, s, zp, qmin, qmax, gscale), (y, gx, gs, gz) in zip(cases, got):
        x = x0.clone().requires_grad_(True)
        yr = FQ.FakeQuantLearnFn.apply(x, s, zp, qmin, qmax, gscale, asym, None)
        yr.backward(gy)
        G.assert_bitwise_f32(y.cpu().numpy(), yr.detach().cpu().numpy(), "y")
        G.assert_bitwise_f32(gx.cpu().numpy(), x.grad.cpu().numpy(), "grad_x")
        assert torch.equal(gs, s.grad), (gs, s.grad)
        if asym:
            assert torch.equal(gz, zp.grad), (gz, zp.grad)
        s.grad = None
        if asym:
            zp.grad = None


def test_multi_misaligned_view():
    """A tensor 4 bytes off 16-byte alignment takes the scalar body inside the launch."""
    xb = (torch.randn(4609, device=DEV) * 0.05).requires_grad_(True)
    gy = torch.randn(4608, device=DEV)
    s1 = nn.Parameter(torch.tensor(0.02, dtype=torch.float64, device=DEV))
    s2 = nn.Parameter(torch.tensor(0.02, dtype=torch.float64, device=DEV))
    gscale = (7 * 4608) ** -0.5
    ys = FQ.lsq_fake_quant_multi([xb[1:], torch.zeros(8, device=DEV)],
                                 [FQ.LsqSpec(s1, 0, -8, 7, gscale, False), FQ.LsqSpec(0.5, 0, -8, 7, 1.0, False)])
    ys[0].backward(gy)
    xr = xb.detach()[1:].clone().requires_grad_(True)
    yr = FQ.FakeQuantLearnFn.apply(xr, s2, 0, -8, 7, gscale, False, None)
    yr.backward(gy)
    G.assert_bitwise_f32(ys[0].detach().cpu().numpy(), yr.detach().cpu().numpy(), "y")
    G.assert_bitwise_f32(xb.grad[1:].cpu().numpy(), xr.grad.cpu().numpy(), "grad_x")
    assert torch.equal(s1.grad, s2.grad)


def test_multi_matches_oracle():
    rng = np.random.default_rng(3)
    xs_np = [rng.standard_normal(n).astype(np.float32) * 0.05 for n in (432, 4608, 1023)]
    gs_np = [rng.standard_normal(x.size).astype(np.float32) for x in xs_np]
    scales = [0.011, 0.02, 0.031]
    xs = [torch.from_numpy(x).to(DEV).requires_grad_(True) for x in xs_np]
    ps = [nn.Parameter(torch.tensor(s, dtype=torch.float64, device=DEV)) for s in scales]
    specs = [FQ.LsqSpec(p, 0, -2, 1, (1 * x.size) ** -0.5, False) for p, x in zip(ps, xs_np)]
    ys = FQ.lsq_fake_quant_multi(xs, specs)
    torch.autograd.backward(ys, [torch.from_numpy(g).to(DEV) for g in gs_np])
    for x_np, g_np, s, x, y, p in zip(xs_np, gs_np, scales, xs, ys, ps):
        yo, gxo, gso, _ = O.lsq_forward_backward(x_np, g_np, s, 0, -2, 1, O.grad_scale(1, x_np.size))
        G.assert_bitwise_f32(y.detach().cpu().numpy(), yo, "y")
        G.assert_bitwise_f32(x.grad.cpu().numpy(), gxo, "grad_x")
        assert abs(float(p.grad) - gso) <= 1e-9 * abs(gso)


def _model():
    torch.manual_seed(0)
    layers = []
    for cin, cout, k in ((3, 16, 3), (16, 32, 3), (32, 32, 1), (32, 64, 3)):
        cv = nn.Conv2d(cin, cout, k, padding=k // 2, bias=False)
        bn = nn.BatchNorm2d(cout)
        bn.running_var.uniform_(0.5, 2.0)
        layers.append(ConvBnReLU(cv, bn, nn.ReLU(), "MinMaxObserver", "UniformQuantizer", "MinMaxObserver",
                                 "UniformQuantizer", True, True, True, 2, 4))
    m = nn.Sequential(*layers).to(DEV)
    for layer in m:   # learnable scales without a calibration pass
        for qm in (layer.weight_quantizer, layer.activation_quantizer):
            qm.mean_abs_x = [0.05]
    activate_learning_qparam(m, use_init=True, model_launches=False)   # per layer; K7 enabled per test
    activate_quantizer(m, model_launches=False)
    return m.to(DEV)   # the new f64 scale Parameters (reference flow: yolov8_qat.py moves the model)


def test_model_hook_equals_per_layer():
    """enable_multi_tensor_weights: the model's output equals the per-layer path bit for
    bit and every gradient (weights, f64 scales) agrees, with one weight launch each way."""
    import copy
    a = _model()
    b = copy.deepcopy(a)
    x = torch.randn(2, 3, 16, 16, device=DEV)
    h = enable_multi_tensor_weights(a)
    try:
        ya = a(x)
    finally:
        h.remove()
    assert all("_weight_stash" not in m.__dict__ for m in a)   # consumed by the forward
    yb = b(x)
    G.assert_bitwise_f32(ya.detach().cpu().numpy(), yb.detach().cpu().numpy(), "model output")
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    pa, pb = dict(a.named_parameters()), dict(b.named_parameters())
    assert pa.keys() == pb.keys()
    # the upstream gradients come through MIOpen's conv backward, whose weight gradient
    # is not run-to-run deterministic: compare to fp32 reordering (the kernels' own
    # bit-identity is test_multi_equals_per_tensor)
    for k in pa:
        assert (pa[k].grad is None) == (pb[k].grad is None), k
        if pa[k].grad is not None:
            torch.testing.assert_close(pa[k].grad, pb[k].grad, rtol=1e-4, atol=1e-6, msg=k)


def test_ineligible_layers_keep_their_path():
    """Observing (calibration) weight quantizers are not batched."""
    m = _model()
    m[0].weight_quantizer.is_learning_scale = False
    n = quantize_weights_multi(list(m))
    assert n == len(m) - 1
    assert "_weight_stash" not in m[0].__dict__
    for layer in m:
        layer.__dict__.pop("_weight_stash", None)
