"""Pin the numpy oracle against the reference goldens (CPU only, no GPU).

The goldens were produced by running the reference itself
(tests/golden/gen_goldens.py); passing here is what makes the oracle a
trustworthy checker for the HIP kernels (tests/test_gpu_parity.py).
"""
import math

import numpy as np
import pytest

from oracle import fakequant_np as O
from tests import goldens as G


@pytest.mark.parametrize("case", G.cases("per_tensor_observe_fq"), ids=lambda c: c["key"])
def test_per_tensor_observe_fq(case):
    x = G.arr(case["x"])
    mn, mx = O.observe_minmax(x, 0, 0)
    assert float(mn) == case["min_val"] and float(mx) == case["max_val"]
    if "raises" in case:
        with pytest.raises(Exception) as ei:
            O.minmax_qparams(mn, mx, case["sym"], case["obs_bits"])
        assert type(ei.value).__name__ == case["raises"]
        return
    s, z = O.minmax_qparams(mn, mx, case["sym"], case["obs_bits"])
    assert (s == case["scale"]) or (math.isnan(s) and math.isnan(case["scale"]))
    assert z == case["zp"]
    qmin, qmax = O.qrange(case["bits"], case["sym"])
    y, q, mask = O.fq_forward(x, s, z, qmin, qmax)
    G.assert_bitwise_f32(y, G.arr(case["y"]), "y")
    G.assert_bitwise_f32(q, G.arr(case["x_int"]), "x_int")
    gx = O.fq_backward_fixed(G.arr(case["g"]), mask, s)
    G.assert_bitwise_f32(gx, G.arr(case["grad_x"]), "grad_x")


@pytest.mark.parametrize("case", G.cases("fixed_fq"), ids=lambda c: c["key"])
def test_fixed_fq(case):
    x = G.arr(case["x"])
    qmin, qmax = O.qrange(case["bits"], case["sym"])
    y, q, mask = O.fq_forward(x, case["scale"], case["zp"], qmin, qmax)
    G.assert_bitwise_f32(y, G.arr(case["y"]), "y")
    G.assert_bitwise_f32(q, G.arr(case["x_int"]), "x_int")
    gx = O.fq_backward_fixed(G.arr(case["g"]), mask, case["scale"])
    G.assert_bitwise_f32(gx, G.arr(case["grad_x"]), "grad_x")


@pytest.mark.parametrize("case", G.cases("per_channel_observe_fq"), ids=lambda c: c["key"])
def test_per_channel(case):
    w = G.arr(case["x"])
    r = O.per_channel_observe_fq(w, case["sym"], case["bits"], case["obs_bits"])
    assert np.array_equal(r["scale"], G.arr(case["scale"]), equal_nan=True)
    assert np.array_equal(r["zp"], G.arr(case["zp"]))
    assert np.array_equal(r["min_val"], G.arr(case["min_val"]))
    assert np.array_equal(r["max_val"], G.arr(case["max_val"]))
    G.assert_bitwise_f32(r["y"], G.arr(case["y"]), "y")
    G.assert_bitwise_f32(r["x_int"], G.arr(case["x_int"]), "x_int")
    gx = O.per_channel_backward_fixed(G.arr(case["g"]), r["mask"], r["scale"])
    G.assert_bitwise_f32(gx, G.arr(case["grad_x"]), "grad_x")


@pytest.mark.parametrize("case", G.cases("learnable_fq"), ids=lambda c: c["key"])
def test_learnable(case):
    x, g = G.arr(case["x"]), G.arr(case["g"])
    qmin, qmax = O.qrange(case["bits"], case["sym"])
    gs = O.grad_scale(qmax, x.size)
    y, gx, gsc, gzp = O.lsq_forward_backward(x, g, case["scale"], case["zp"], qmin, qmax, gs,
                                             learn_zp=not case["sym"])
    G.assert_bitwise_f32(y, G.arr(case["y"]), "y")
    G.assert_bitwise_f32(gx, G.arr(case["grad_x"]), "grad_x")
    # reference sums in fp32 -> tolerance (SURVEY §8d parity gates: <=1e-4 relative)
    assert gsc == pytest.approx(case["scale_grad"], rel=1e-4, abs=1e-9)
    if not case["sym"]:
        assert gzp == pytest.approx(case["zp_grad"], rel=1e-4, abs=1e-9)


@pytest.mark.parametrize("case", G.cases("learnable_fq_calib"), ids=lambda c: c["key"])
def test_learnable_calib_grad_scale_tensor(case):
    """Per-channel calib_grad_scale tensor (utils/estimate_bn.py:136): the effective
    gradient factor is (qmax*numel)^-1/2 * sum(calib) (autograd's sum_to onto the 0-dim
    scale, uniform.py:47-53,252-253); the reference multiplies and sums in fp32."""
    x, g = G.arr(case["x"]), G.arr(case["g"])
    qmin, qmax = O.qrange(case["bits"], case["sym"])
    calib = float(G.arr(case["calib"]).astype(np.float64).sum())
    y, gx, gsc, gzp = O.lsq_forward_backward(x, g, case["scale"], case["zp"], qmin, qmax,
                                             O.grad_scale(qmax, x.size, calib), learn_zp=not case["sym"])
    G.assert_bitwise_f32(y, G.arr(case["y"]), "y")
    G.assert_bitwise_f32(gx, G.arr(case["grad_x"]), "grad_x")
    assert gsc == pytest.approx(case["scale_grad"], rel=1e-4, abs=1e-9)
    if not case["sym"]:
        assert gzp == pytest.approx(case["zp_grad"], rel=1e-4, abs=1e-9)


def test_asym_learnable_int_zp_raises_in_reference():
    (c,) = G.cases("asym_learnable_int_zp")
    assert c["raises"] == "TypeError"


@pytest.mark.parametrize("case", G.cases("manager_sequence"), ids=lambda c: c["key"])
def test_manager_sequence(case):
    """QuantizationManager calibrate -> observe+quantize -> learn-init (qm.py:55-114)."""
    bits, sym = case["bits"], case["sym"]
    mn, mx = 0, 0
    stats = []
    for k in case["xs"]:
        x = G.arr(k)
        stats.append(O.collect_stats(x))
        mn, mx = O.observe_minmax(x, mn, mx)
    cal = case["calib"]
    assert (mn, mx) == (cal["min_val"], cal["max_val"])
    s, z = O.minmax_qparams(mn, mx, sym, 8)  # observer is always 8-bit (qm.py:42)
    assert s == cal["scale"] and z == cal["zero_point"]
    np.testing.assert_allclose([t[0] for t in stats], cal["mean_abs_x"], rtol=1e-6)
    np.testing.assert_allclose([t[1] for t in stats], cal["mean_x"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose([t[2] for t in stats], cal["std"], rtol=1e-6)
    # observe + quantize in the same call
    xo = G.arr(case["x_oq"])
    mn, mx = O.observe_minmax(xo, mn, mx)
    s, z = O.minmax_qparams(mn, mx, sym, 8)
    assert s == case["observe_quantize"]["scale"]
    qmin, qmax = O.qrange(bits, sym)
    y, _, _ = O.fq_forward(xo, s, z, qmin, qmax)
    G.assert_bitwise_f32(y, G.arr(case["y_oq"]), "y_oq")
    init = O.init_scale_for_learning([t[0] for t in stats] + [O.collect_stats(xo)[0]], bits)
    assert init == pytest.approx(case["init_scale"], rel=1e-6)
    if "learn_raises" in case:
        assert case["learn_raises"] == "TypeError" and not sym
        return
    x4, g4 = G.arr(case["x4"]), G.arr(case["g4"])
    s_ref = case["init_scale"]
    gs = O.grad_scale(qmax, x4.size)
    y4, gx4, gsc, _ = O.lsq_forward_backward(x4, g4, s_ref, 0, qmin, qmax, gs)
    G.assert_bitwise_f32(y4, G.arr(case["y4"]), "y4")
    G.assert_bitwise_f32(gx4, G.arr(case["gx4"]), "gx4")
    assert gsc == pytest.approx(case["scale_grad"], rel=1e-4)


@pytest.mark.parametrize("case", G.cases("act_fq"), ids=lambda c: c["key"])
def test_act_fq(case):
    """Fused activation + activation fake quant (K5): bit-exact for ReLU and SiLU (torch's
    CPU silu restated with its two exps, oracle/silu_ref.c)."""
    c = G.arr(case["x"])
    g = G.arr(case["g"])
    qmin, qmax = O.qrange(case["bits"], case["sym"])
    a = O.act_forward(c, case["act"])
    if case["mode"] == "observe":
        s, z = O.minmax_qparams(*O.observe_minmax(a), case["sym"], 8)
        assert (s, z) == (case["scale"], case["zp"])
    else:
        s, z = case["scale"], case["zp"]
    if case["mode"] == "learn":
        y, gx, gs, _ = O.lsq_forward_backward(a, g, s, 0, qmin, qmax, O.grad_scale(qmax, c.size))
        assert abs(gs - case["scale_grad"]) <= 1e-4 * max(1e-3, abs(case["scale_grad"]))
    else:
        y, _, m = O.fq_forward(a, s, z, qmin, qmax)
        gx = O.fq_backward_fixed(g, m, s)
    gc = O.act_backward(gx, c, case["act"])
    G.assert_bitwise_f32(y, G.arr(case["y"]), "y")
    G.assert_bitwise_f32(gc, G.arr(case["grad_x"]), "grad_c")


@pytest.mark.parametrize("case", [c for c in G.cases("fused_layer") if c["act"]], ids=lambda c: c["key"])
@pytest.mark.parametrize("mode", ["observe", "learn"])
def test_fused_layer_activation(case, mode):
    """The fused layers' F.relu / F.silu + quantize_out on the reference's own
    pre-activation (modules/fused.py:133, fake_quantize.py:49-50): y and the gradient
    with respect to the pre-activation bit-exact.  fz1 / fz9 (SiLU, 1296 and 120
    elements) have 16 / 24 elements on torch's scalar (glibc expf) path."""
    if mode not in case:
        pytest.skip("asymmetric layer: no learnable mode in the reference")
    rec = case[mode]
    pre, g = G.arr(rec["pre"]), G.arr(rec["g"])
    a = O.act_forward(pre, case["act"])
    qmin, qmax = O.qrange(case["bits_a"], case["a_sym"])
    if mode == "observe":
        s, z = O.minmax_qparams(*O.observe_minmax(a), case["a_sym"], 8)
        assert (s, z) == (rec["act_qp"]["scale"], rec["act_qp"]["zp"])
        y, _, m = O.fq_forward(a, s, z, qmin, qmax)
        gx = O.fq_backward_fixed(g, m, s)
    else:
        y, gx, gs, _ = O.lsq_forward_backward(a, g, rec["init_scale_a"], 0, qmin, qmax,
                                              O.grad_scale(qmax, a.size))
        assert gs == pytest.approx(rec["scale_grad_a"], rel=1e-4)
    G.assert_bitwise_f32(y, G.arr(rec["y"]), "y")
    G.assert_bitwise_f32(O.act_backward(gx, pre, case["act"]), G.arr(rec["grad_pre"]), "grad_pre")


@pytest.mark.parametrize("case", G.cases("lsq_fake_quantize"), ids=lambda c: c["key"])
def test_lsq_fake_quantize(case):
    """LSQFakeQuantize learnable fwd+bwd (per-channel axis 1 / per-tensor, x5000 for acts)."""
    x, g = G.arr(case["x"]), G.arr(case["g"])
    s, z = G.arr(case["scale"]).reshape(-1), G.arr(case["zp"]).reshape(-1)
    gsc = O.lsq_module_grad_scale(x.shape, case["qmax"], case["per_channel"], case["config_act"])
    if case["per_channel"]:
        y, gx, gs, gz = O.pc_lsq_forward_backward(x, g, s, z, case["qmin"], case["qmax"], gsc, axis=1)
    else:
        y, gx, gs0, gz0 = O.lsq_forward_backward(x, g, float(s[0]), float(z[0]), case["qmin"], case["qmax"],
                                                 gsc, learn_zp=True)
        gs, gz = np.array([gs0]), np.array([gz0])
    G.assert_bitwise_f32(y, G.arr(case["y"]), "y")
    G.assert_bitwise_f32(gx, G.arr(case["grad_x"]), "grad_x")
    np.testing.assert_allclose(gs, G.arr(case["scale_grad"]).reshape(-1), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(gz, G.arr(case["zp_grad"]).reshape(-1), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("case", G.cases("learnable_fq_sym_tensor_zp"), ids=lambda c: c["key"])
def test_learnable_sym_tensor_zp(case):
    """Symmetric learnable quantize with a gradient-requiring tensor zero point
    (uniform.py:47-56: no zero_point_rounding / ScaleGradient on zp in the symmetric
    branch): zp as given; its gradient sum g*s*(mask-1) without gscale."""
    x, g = G.arr(case["x"]), G.arr(case["g"])
    qmin, qmax = O.qrange(case["bits"], True)
    y, gx, gsc, gzp = O.lsq_forward_backward(x, g, case["scale"], case["zp"], qmin, qmax,
                                             O.grad_scale(qmax, x.size), learn_zp=2)
    G.assert_bitwise_f32(y, G.arr(case["y"]), "y")
    G.assert_bitwise_f32(gx, G.arr(case["grad_x"]), "grad_x")
    # the reference sums ~3K fp32 terms in fp32 (error ~1e-6 absolute; these gradients
    # cancel down to 1e-3..1e-2): 1e-4 relative or 3e-6 absolute
    assert gsc == pytest.approx(case["scale_grad"], rel=1e-4, abs=3e-6)
    assert gzp == pytest.approx(case["zp_grad"], rel=1e-4, abs=3e-6)
