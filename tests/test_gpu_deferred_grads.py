"""Deferred learnable-qparam gradient fold (K4d: vsiq_act_lsq_bwd_part_f32 +
vsiq_lsq_fold_multi; quantizers/deferred.py).  grad_x bit for bit equal to K4's, the
folded scale / zero-point gradients equal to K4's in-kernel fold to float64 summation
order and to the oracle's f64 closed form (uniform.py:47-56, ScaleGradient :242-255);
through autograd, a fused QAT model's step equals the per-call path."""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

import vsiquantization_amd as V
from vsiquantization_amd import _hip as H
from vsiquantization_amd import fakequant as FQ
from vsiquantization_amd.quantizers import deferred as D
from oracle import fakequant_np as O
from tests import goldens as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("act", [None, "relu"])
@pytest.mark.parametrize("learn_zp", [False, True])
def test_part_and_fold_equal_k4_and_oracle(act, learn_zp):
    rng = np.random.default_rng(17 + int(learn_zp))
    # + the one-round gated K4d form's sizes (k4d_one_round: 4.7M..9.4M elements, C4's 6.6M layers)
    sizes = ([1, 7, 1000, 65536, 1 << 20, 3 * (1 << 20) + 3, 4_718_592, 6_553_600 + 5, 9_437_184]
             + [4096 + 13 * k for k in range(66)])   # 75 calls
    qmin, qmax = (0, 15) if learn_zp else (-8, 7)
    calls = []
    for n in sizes:
        x = (rng.standard_normal(n) * 0.3).astype(np.float32)
        g = rng.standard_normal(n).astype(np.float32)
        s, z = float(rng.uniform(0.01, 0.1)), (float(rng.integers(3, 12)) + 0.3 if learn_zp else 0.0)
        gscale = (qmax * n) ** -0.5
        calls.append((x, g, s, z, gscale))
    folds = []
    for x, g, s, z, gscale in calls:
        xd, gd = torch.from_numpy(x).to(DEV), torch.from_numpy(g).to(DEV)
        sd = torch.tensor(s, dtype=torch.float64, device=DEV)
        zd = torch.tensor(z, dtype=torch.float64, device=DEV) if learn_zp else 0.0
        gx_ref, grads_ref = FQ.lsq_backward(gd, xd, sd, zd, qmin, qmax, gscale, learn_zp, act=act)
        e = D._Fold()
        e.nrec = int(H.lib().vsiq_lsq_part_records(H.c_i64(x.size)))
        e.records = torch.full((2 * e.nrec,), float("nan"), dtype=torch.float64, device=DEV)
        gx, e.zd, e.zh = D.lsq_backward_part(gd, xd, sd, zd, qmin, qmax, learn_zp, act, e.records)
        e.gscale, e.qmin, e.qmax, e.learn_zp = gscale, qmin, qmax, learn_zp
        e.out = torch.empty(2, dtype=torch.float64, device=DEV)
        e.keep = (sd, zd)
        folds.append((e, gx, gx_ref, grads_ref, x, g, s, z, gscale))
    D.fold([f[0] for f in folds])
    torch.cuda.synchronize()
    for e, gx, gx_ref, grads_ref, x, g, s, z, gscale in folds:
        assert torch.equal(gx.view(torch.int32), gx_ref.view(torch.int32))
        got, ref = e.out.cpu().numpy(), grads_ref.cpu().numpy()
        np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-300)
        if act is None:
            _, gxo, gso, gzo = O.lsq_forward_backward(x, g, s, z, qmin, qmax, gscale, learn_zp=learn_zp)
            G.assert_bitwise_f32(gx.cpu().numpy(), gxo, "grad_x")
            np.testing.assert_allclose(got[0], gso, rtol=1e-9, atol=1e-300)
            if learn_zp:
                np.testing.assert_allclose(got[1], gzo, rtol=1e-9, atol=1e-300)


def _model(act_learn_zp=False):
    from vsiquantization_amd.modules.fused import ConvBnReLU
    from vsiquantization_amd.utils.quantize_manager import (activate_learning_qparam, activate_quantizer,
                                                            calibrate_qat_model, data_calib)
    torch.manual_seed(0)
    layers = []
    for cin, cout in ((3, 16), (16, 32), (32, 32)):
        bn = nn.BatchNorm2d(cout)
        bn.running_var.uniform_(0.5, 2.0)
        layers.append(ConvBnReLU(nn.Conv2d(cin, cout, 3, padding=1, bias=False), bn, nn.ReLU(),
                                 "MinMaxObserver", "UniformQuantizer", "MinMaxObserver", "UniformQuantizer",
                                 True, True, True, 4, 4))
    model = nn.Sequential(*layers).to(DEV)
    gen = torch.Generator().manual_seed(1)
    loader = [(torch.randint(0, 256, (4, 3, 32, 32), generator=gen, dtype=torch.uint8), None) for _ in range(2)]
    calibrate_qat_model(model, loader, data_calib, DEV)
    activate_learning_qparam(model, model_launches=False)   # the per-call path; hooks enabled per test
    activate_quantizer(model, model_launches=False)
    model.eval()
    return model


@pytest.mark.parametrize("multi_weights", [False, True])
def test_model_step_deferred_equals_per_call(multi_weights):
    """A fused QAT model's forward + backward with enable_deferred_qparam_grads: output,
    grad of the input and conv biases bit for bit; the activation quantizers' f64 scale
    gradients within 1e-12 of the per-call path (float64 summation order); conv weights
    and weight-quantizer scales within MIOpen's wgrad nondeterminism (1e-5); nothing left
    pending."""
    a = _model()
    b = copy.deepcopy(a)
    handles = [V.enable_deferred_qparam_grads(a)]
    if multi_weights:
        handles += [V.enable_multi_tensor_weights(a), V.enable_multi_tensor_weights(b)]
    x = torch.rand(4, 3, 32, 32, device=DEV)
    outs = []
    for m in (a, b):
        xi = x.clone().requires_grad_(True)
        y = m(xi)
        y.square().mean().backward()
        outs.append((y.detach(), xi.grad))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    for (na, pa), (nb, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert na == nb
        if pa.grad is None:
            assert pb.grad is None, na
            continue
        if "activation_quantizer" in na or "input_quantizer" in na:
            np.testing.assert_allclose(pa.grad.cpu().numpy(), pb.grad.cpu().numpy(), rtol=1e-12, atol=1e-300,
                                       err_msg=na)
        elif na.endswith("weight") or "weight_quantizer" in na:
            # the weight quantizer's gradient is computed from MIOpen's weight-gradient
            # convolution, which is not bit-reproducible run to run (~1e-7 relative)
            torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-5, atol=1e-12, msg=na)
        else:
            assert torch.equal(pa.grad, pb.grad), na
    assert D.pending_count() == 0
    for h in handles:
        h.remove()


def test_model_step_deferred_graph_replay_equals_eager():
    from vsiquantization_amd.utils.graph import GraphedStep
    m = _model()
    h = V.enable_deferred_qparam_grads(m)
    x = torch.rand(4, 3, 32, 32, device=DEV)
    params = [p for p in m.parameters() if p.requires_grad]

    def step():
        y = m(x)
        y.square().mean().backward()
        return y

    for p in params:
        p.grad = None
    y_ref = step().detach().clone()
    g_ref = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    gs = GraphedStep(step, grads_of=params)
    for _ in range(2):
        y = gs()
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)
    for n, p in m.named_parameters():
        if n in g_ref:
            if n.endswith("conv_fuse.weight") or n.endswith("weight_quantizer.scale"):
                torch.testing.assert_close(p.grad, g_ref[n], rtol=1e-5, atol=1e-12, msg=n)
            else:
                assert torch.equal(p.grad, g_ref[n]), n
    h.remove()


def test_second_use_in_one_forward_takes_per_call_path():
    """A manager called twice in one forward: the first call uses the bundle, the second
    the per-call path; gradients equal the per-call path's."""
    q = V.QuantizationManager("UniformQuantizer", "MinMaxObserver", 8, True, is_learning_scale=True)
    q.scale = nn.Parameter(torch.tensor(0.05, dtype=torch.float64, device=DEV))
    x = torch.randn(1000, device=DEV, requires_grad=True)
    ref = copy.deepcopy(q)
    D.bundle_qparams([q])
    (q.quantize(x) + q.quantize(x * 2)).sum().backward()
    x2 = x.detach().clone().requires_grad_(True)
    (ref.quantize(x2) + ref.quantize(x2 * 2)).sum().backward()
    torch.cuda.synchronize()
    assert torch.equal(x.grad, x2.grad)
    np.testing.assert_allclose(float(q.scale.grad), float(ref.scale.grad), rtol=1e-12)
    assert D.pending_count() == 0


@pytest.mark.parametrize("act_learn_zp", [False, True])
def test_deferred_cpp_node_equals_python_function(act_learn_zp, monkeypatch):
    """The records-only backward as the C++ node (FqLearnDeferredBackward + deferred_fold,
    the default) and as the Python DeferredLearnFn (VSIQ_TORCH_EXT=0): the same kernels and
    arguments, so output, input gradient and every qparam gradient bit for bit, and
    nothing left pending in either table."""
    from vsiquantization_amd import _hip as H
    base = _model()
    if act_learn_zp:   # the last layer's activation quantizer: asymmetric LSQ, learned zero point
        qm = base[2].activation_quantizer
        qm.quantizer = V.LSQQuantizer(4, False)
        qm.zero_point = nn.Parameter(torch.tensor(3.0, dtype=torch.float64, device=DEV))
    x = torch.rand(4, 3, 32, 32, device=DEV)
    res = []
    for ext in (True, False):
        monkeypatch.setattr(H, "torch_ext_enabled", lambda e=ext: e)
        m = copy.deepcopy(base)
        h = V.enable_deferred_qparam_grads(m)
        for _ in range(2):   # two steps: the second runs on a new forward generation
            for p in m.parameters():
                p.grad = None
            xi = x.clone().requires_grad_(True)
            y = m(xi)
            y.square().mean().backward()
        torch.cuda.synchronize()
        res.append((y.detach(), xi.grad, {n: p.grad.clone() for n, p in m.named_parameters()
                                          if p.grad is not None and "quantizer" in n}))
        assert D.pending_count() == 0
        h.remove()
    monkeypatch.undo()
    (ya, ga, qa), (yb, gb, qb) = res
    assert torch.equal(ya, yb) and torch.equal(ga, gb)
    assert qa.keys() == qb.keys() and len(qa) >= 6
    if act_learn_zp:
        assert "2.activation_quantizer.zero_point" in qa
    for n in qa:
        if "weight_quantizer" in n:   # from MIOpen's weight-gradient conv (not bit-reproducible)
            torch.testing.assert_close(qa[n], qb[n], rtol=1e-5, atol=1e-12, msg=n)
        else:
            assert torch.equal(qa[n], qb[n]), n


@pytest.mark.parametrize("ext", [True, False])
def test_orphaned_pending_folds_dropped_next_forward(ext, monkeypatch):
    """torch.autograd.grad with respect to the input only never reaches the bundle node, so
    its records-only backwards stay pending; they are dropped at the next forward but one
    (one generation of slack), in the C++ table and in the Python one alike, and a normal
    step afterwards leaves nothing pending."""
    from vsiquantization_amd import _hip as H
    monkeypatch.setattr(H, "torch_ext_enabled", lambda e=ext: e)
    m = _model()
    h = V.enable_deferred_qparam_grads(m)
    x = torch.rand(2, 3, 32, 32, device=DEV, requires_grad=True)
    (gx,) = torch.autograd.grad(m(x).square().mean(), x)
    assert D.pending_count() == 3   # one per activation quantizer
    with torch.no_grad():
        m(x)
        m(x)
    assert D.pending_count() == 0
    m(x).square().mean().backward()
    torch.cuda.synchronize()
    assert D.pending_count() == 0
    h.remove()


def test_deepcopy_of_enabled_model_defers_its_own_managers():
    """A deep copy of a model with K7 + K4d enabled (an EMA or teacher copy) runs the same
    model-level launches on ITS OWN layers and managers: the same output and activation
    scale gradients bit for bit as the original, nothing left pending, and the original's
    managers untouched by the copy's forward."""
    m = _model()
    hs = [V.enable_deferred_qparam_grads(m), V.enable_multi_tensor_weights(m)]
    c = copy.deepcopy(m)
    x = torch.rand(2, 3, 32, 32, device=DEV)
    res = []
    for mod in (m, c):
        for p in mod.parameters():
            p.grad = None
        y = mod(x)
        assert all("_deferred_qparams" not in qm.__dict__ for qm in D._managers(m))
        y.square().mean().backward()
        torch.cuda.synchronize()
        res.append((y.detach(), {n: p.grad for n, p in mod.named_parameters()
                                 if p.grad is not None and "activation_quantizer" in n}))
    assert D.pending_count() == 0
    assert torch.equal(res[0][0], res[1][0])
    assert res[0][1].keys() == res[1][1].keys() and len(res[0][1]) == 3
    for n in res[0][1]:
        assert torch.equal(res[0][1][n], res[1][1][n]), n
    for h in hs:
        h.remove()


def _edge_values(s):
    """x and g values at and just past the K4 fast path's bounds for scale s (k_body.cuh
    lsq_fast_ok4x: |x| in [max(2^-40, s 2^-61), min(2^63, s 2^61)], in-range |g| in
    [2^-40, 2^63], or zero), plus subnormals and zeros of both signs."""
    f = np.float32
    up = lambda v: np.nextafter(f(v), f(np.inf))     # noqa: E731
    dn = lambda v: np.nextafter(f(v), f(0))          # noqa: E731
    lo, hi = max(2.0 ** -40, s * 2.0 ** -61), min(2.0 ** 63, s * 2.0 ** 61)
    xs = [0.0, -0.0, lo, dn(lo), hi, up(hi), -hi, 2.0 ** -40, dn(2.0 ** -40), 2.0 ** 63, up(2.0 ** 63),
          1e-45, -1e-40, s * 3.5, -s * 7.5, s * 0.5, s * 1.5]
    gs = [0.0, -0.0, 2.0 ** -40, dn(2.0 ** -40), 2.0 ** 20, -(2.0 ** 20), 1e-45, -3e-39, 0.7, -1.3, 5.0]
    return np.array(xs, dtype=np.float32), np.array(gs, dtype=np.float32)


# ste_fast_s admits the closed range [2^-60, 2^60]: both ends and the floats just outside
@pytest.mark.parametrize("s", [float(np.nextafter(np.float32(2.0 ** -60), np.float32(0))), 2.0 ** -60,
                               2.0 ** -59.5, 1e-3, 0.03, 1.0, 2.0 ** 40, 2.0 ** 59.5, 2.0 ** 60,
                               float(np.nextafter(np.float32(2.0 ** 60), np.float32(np.inf)))])
@pytest.mark.parametrize("act", [None, "relu"])
def test_fast_path_bounds_k4_k4d(s, act):
    """Elements at and past every bound of the K4 / K4d fast-path test, in random groups of
    four among ordinary values (so groups take the fast path, the general fast division or
    IEEE): grad_x bit for bit equal to the oracle (no act) and between K4 and K4d, the scale
    gradient to f64 order (bounded by the sum of the terms' magnitudes)."""
    rng = np.random.default_rng(int(s * 1e3) % 9973 + (act is not None))
    ex, eg = _edge_values(s)
    n = 4 * 2048 + 3
    x = (rng.standard_normal(n) * 4 * s).astype(np.float32)
    g = rng.standard_normal(n).astype(np.float32)
    idx = rng.choice(n, size=600, replace=False)
    x[idx] = ex[rng.integers(0, ex.size, idx.size)]
    idx = rng.choice(n, size=600, replace=False)
    g[idx] = eg[rng.integers(0, eg.size, idx.size)]
    qmin, qmax, gscale = -8, 7, 0.37
    xd, gd = torch.from_numpy(x).to(DEV), torch.from_numpy(g).to(DEV)
    sd = torch.tensor(s, dtype=torch.float64, device=DEV)
    gx4, grads4 = FQ.lsq_backward(gd, xd, sd, 0.0, qmin, qmax, gscale, False, act=act)
    e = D._Fold()
    e.nrec = int(H.lib().vsiq_lsq_part_records(H.c_i64(n)))
    e.records = torch.full((2 * e.nrec,), float("nan"), dtype=torch.float64, device=DEV)
    gxd, e.zd, e.zh = D.lsq_backward_part(gd, xd, sd, 0.0, qmin, qmax, False, act, e.records)
    e.gscale, e.qmin, e.qmax, e.learn_zp = gscale, qmin, qmax, False
    e.out = torch.empty(2, dtype=torch.float64, device=DEV)
    D.fold([e])
    torch.cuda.synchronize()
    assert torch.equal(gx4.view(torch.int32), gxd.view(torch.int32))
    bound = 1e-13 * 2 * float(np.abs(g.astype(np.float64)).sum()) * (qmax + 2) * gscale
    g4, gd_ = float(grads4[0]), float(e.out[0])

    def close(a, b, rel):   # NaN where the terms hold 0 * inf (x / s / s overflows at tiny s), as in torch
        return (np.isnan(a) and np.isnan(b)) or abs(a - b) <= bound + rel * abs(b)

    assert close(g4, gd_, 1e-12), (g4, gd_)
    if act is None:
        _, gxo, gso, _ = O.lsq_forward_backward(x, g, s, 0.0, qmin, qmax, gscale)
        G.assert_bitwise_f32(gx4.cpu().numpy(), gxo, "grad_x")
        assert close(g4, gso, 1e-9), (g4, gso)
