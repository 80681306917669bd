"""K5: fused ReLU/SiLU + activation fake quant on MI355X, through the C ABI.

Bars: ReLU and SiLU bit-exact against the reference goldens and the oracle (y, grad
w.r.t. the pre-activation; SiLU is torch's CPU silu bit for bit, both exps and the
chunk layout, oracle/silu_ref.c); scale gradients <= 1e-4 (reference fp32 sums) /
1e-9 (oracle f64).  The fused module path equals the unfused composition bitwise.
"""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import vsiquantization_amd as V
from vsiquantization_amd import _hip as H
from vsiquantization_amd import fakequant as FQ
from vsiquantization_amd.modules.fused import ConvBnReLU
from vsiquantization_amd.quantizers.fake_quantize import FakeQuantize
from oracle import fakequant_np as O
from tests import goldens as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(autouse=True)
def _golden_silu_host():
    """SiLU as on the goldens' reference host (tests/goldens.py: GOLDEN_SILU_REF)."""
    H.set_silu_reference(*G.GOLDEN_SILU_REF)
    yield
    H.set_silu_reference()


def cu(a, grad=False):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    return t.requires_grad_(grad) if grad else t


def npy(t):
    return t.detach().cpu().numpy()


def _check(act, got_y, want_y, got_g, want_g, scale=None):
    G.assert_bitwise_f32(got_y, want_y, "y")
    G.assert_bitwise_f32(got_g, want_g, "grad_c")


def REF():
    """The reference CPU layout the product reproduces SiLU for (pinned above)."""
    return H.silu_reference()


@pytest.mark.parametrize("case", G.cases("act_fq"), ids=lambda c: c["key"])
def test_golden_act_fq(case):
    act, sym, bits = case["act"], case["sym"], case["bits"]
    q = V.UniformQuantizer(bits, sym)
    c = cu(G.arr(case["x"]), grad=True)
    if case["mode"] == "observe":
        qp, _ = FQ.observe_tensor(c.detach(), symmetric=sym, act=act)
        qph = npy(qp)
        assert (qph[H.QP_SCALE], qph[H.QP_ZP]) == (case["scale"], case["zp"])
        assert (qph[H.QP_MIN], qph[H.QP_MAX]) == (case["min_val"], case["max_val"])
        y = FQ.FakeQuantFixedFn.apply(c, None, None, q.qmin, q.qmax, qp, act)
    elif case["mode"] == "fixed":
        y = q.quantize(c, case["scale"], case["zp"], False, act=act)
    else:
        s = torch.nn.Parameter(torch.tensor(case["scale"], dtype=torch.float64, device=DEV))
        y = q.quantize(c, s, 0, True, act=act)
    y.backward(cu(G.arr(case["g"])))
    _check(act, npy(y), G.arr(case["y"]), npy(c.grad), G.arr(case["grad_x"]), case["scale"])
    if case["mode"] == "learn":
        assert abs(float(s.grad) - case["scale_grad"]) <= 1e-4 * max(1e-3, abs(case["scale_grad"]))


@pytest.mark.parametrize("act", ["relu", "silu"])
@pytest.mark.parametrize("n", [1, 5, 1000, 262_147, 3_000_000])
def test_act_fixed_vs_oracle(act, n):
    rng = np.random.default_rng(n)
    c = (rng.standard_normal(n) * 2).astype(np.float32)
    g = rng.standard_normal(n).astype(np.float32)
    if n > 8:
        c[:6] = [-0.0, 0.0, np.nan, np.inf, -np.inf, 1e-40]
    qmin, qmax = 0, 255
    y, mask, _ = FQ.fake_quant(cu(c), 0.021, 3, qmin, qmax, want_mask=True, act=act)
    gc = FQ.ste_backward(cu(g), mask, 0.021, pre=cu(c), act=act)
    a = O.act_forward(c, act, REF())
    yo, _, mo = O.fq_forward(a, 0.021, 3, qmin, qmax)
    go = O.act_backward(O.fq_backward_fixed(g, mo, 0.021), c, act, REF())
    assert np.array_equal(G.unpack_mask(npy(mask), 1, n)[0], mo)
    _check(act, npy(y), yo, npy(gc), go, 0.021)


@pytest.mark.parametrize("act", ["relu", "silu"])
def test_act_observe_vs_oracle(act):
    rng = np.random.default_rng(7)
    c = (rng.standard_normal(2_000_003) * 3).astype(np.float32)
    qp, st = FQ.observe_tensor(cu(c), symmetric=False, act=act)
    a = O.act_forward(c, act, REF())
    mn, mx = O.observe_minmax(a)
    s, z = O.minmax_qparams(mn, mx, False, 8)
    qph, sth = npy(qp), npy(st)
    assert (qph[H.QP_SCALE], qph[H.QP_ZP]) == (s, z)
    assert (qph[H.QP_MIN], qph[H.QP_MAX]) == (mn, mx)
    want = float(np.float32(np.sum(np.abs(a), dtype=np.float64) / a.size))
    assert abs(sth[H.ST_MEANABS] - want) <= 1e-6 * want
    assert sth[H.ST_N] == c.size


@pytest.mark.parametrize("act", ["relu", "silu"])
def test_act_learnable_c3_size(act):
    rng = np.random.default_rng(11)
    n = 512 * 3 * 64 * 64
    c = rng.standard_normal(n).astype(np.float32)
    g = rng.standard_normal(n).astype(np.float32)
    q = V.UniformQuantizer(8, True)
    s = torch.nn.Parameter(torch.tensor(0.03, dtype=torch.float64, device=DEV))
    cg = cu(c, grad=True)
    y = q.quantize(cg, s, 0, True, act=act)
    y.backward(cu(g))
    a = O.act_forward(c, act, REF())
    yo, gxo, gso, _ = O.lsq_forward_backward(a, g, 0.03, 0, q.qmin, q.qmax, O.grad_scale(q.qmax, n))
    _check(act, npy(y), yo, npy(cg.grad), O.act_backward(gxo, c, act, REF()))
    assert abs(float(s.grad) - gso) <= 1e-9 * abs(gso)


def _conv_bn_relu(seed, act, a_sym=False):
    torch.manual_seed(seed)
    cv = nn.Conv2d(16, 32, 3, padding=1, bias=False)
    bn = nn.BatchNorm2d(32)
    bn.running_mean.uniform_(-0.2, 0.2)
    bn.running_var.uniform_(0.5, 2.0)
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.uniform_(-0.1, 0.1)
    m = ConvBnReLU(cv, bn, nn.ReLU() if act == "relu" else nn.SiLU(), "MinMaxObserver",
                   "UniformQuantizer", "MinMaxObserver", "UniformQuantizer", True, a_sym,
                   True, 8, 8)
    return m.to(DEV)


@pytest.mark.parametrize("act", ["relu", "silu"])
@pytest.mark.parametrize("phase", ["calibrate", "observe_quantize", "learn"])
def test_fused_layer_equals_unfused(act, phase):
    """ConvBnReLU.forward hands the pre-activation to the activation quantizer (K5);
    the result must equal the reference's order (activation, then quantize_out)."""
    # learnable asymmetric UniformQuantizer raises in the reference (int zp): symmetric there
    fused = _conv_bn_relu(3, act, a_sym=phase == "learn")
    for qm in (fused.weight_quantizer, fused.activation_quantizer):
        qm.is_learning_scale, qm.is_observer_qparam, qm.is_quantize = False, True, phase != "calibrate"
    if phase == "learn":
        x0 = torch.randn(8, 16, 20, 20, device=DEV)
        fused(x0)
        for qm in (fused.weight_quantizer, fused.activation_quantizer):
            qm.is_learning_scale, qm.is_quantize = True, True
            qm.init_scaling_factor_for_learning()
            qm.make_learn_qparameter()
    ref = copy.deepcopy(fused)
    x = torch.randn(8, 16, 20, 20, device=DEV)
    xf, xr = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    yf = fused(xf)
    yr = FakeQuantize.forward(ref, xr)          # conv -> F.relu/F.silu -> quantize_out
    g = torch.randn_like(yf)
    yf.backward(g)
    yr.backward(g)
    s = fused.activation_quantizer.scale
    scale = float(s.detach().reshape(-1)[0]) if isinstance(s, torch.Tensor) else float(s)
    _check(act, npy(yf), npy(yr), npy(xf.grad), npy(xr.grad), scale)
    if phase != "learn":
        assert fused.activation_quantizer.observer.min_val == ref.activation_quantizer.observer.min_val
        assert fused.activation_quantizer.observer.max_val == ref.activation_quantizer.observer.max_val
        af, ar = fused.activation_quantizer.mean_abs_x, ref.activation_quantizer.mean_abs_x
        assert np.allclose(af, ar, rtol=1e-6)
    else:
        gf = float(fused.activation_quantizer.scale.grad)
        gr = float(ref.activation_quantizer.scale.grad)
        assert abs(gf - gr) <= 1e-9 * abs(gr)
        # the weight gradient comes from MIOpen's backward-weights (atomic reductions,
        # not run-to-run deterministic): toleranced even for ReLU
        G.assert_close_f32(npy(fused.conv_fuse.weight.grad), npy(ref.conv_fuse.weight.grad),
                           "dW", rtol=1e-4, atol=1e-4)


def test_act_requires_pre_activation():
    g = torch.randn(64, device=DEV)
    _, mask, _ = FQ.fake_quant(g, 0.1, 0, -128, 127, want_mask=True)
    with pytest.raises(H.VsiqError):
        FQ.ste_backward(g, mask, 0.1, pre=torch.randn(64), act="relu")   # CPU pre-activation
    with pytest.raises(ValueError):
        FQ.fake_quant(g, 0.1, 0, -128, 127, act="gelu")
