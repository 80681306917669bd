"""HIP kernels vs the reference goldens and the numpy oracle (MI355X only).

Every test goes through the C ABI (vsiquantization_amd._hip -> _vsiq_hip.so).
Bars: integer codes and fp32 outputs bit-exact (y, x_int, grad_x);
scale / zero-point gradients <= 1e-4 relative to the reference's fp32 sums and
<= 1e-9 relative to the oracle's float64 closed form.
"""
import math

import numpy as np
import pytest
import torch

import vsiquantization_amd as V
from vsiquantization_amd import _hip as H
from vsiquantization_amd import fakequant as FQ
from oracle import fakequant_np as O
from tests import goldens as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def cu(a, grad=False):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    return t.requires_grad_(grad) if grad else t


def npy(t):
    return t.detach().cpu().numpy()


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    H.lib()   # raises if the HIP library is missing: no silent fallback


# --------------------------------------------------------------------------- goldens
@pytest.mark.parametrize("case", G.cases("per_tensor_observe_fq"), ids=lambda c: c["key"])
def test_golden_per_tensor_observe_fq(case):
    x = cu(G.arr(case["x"]))
    obs = V.MinMaxObserver(case["sym"], case["obs_bits"])
    if "raises" in case:
        with pytest.raises(Exception) as ei:
            obs.forward(x)
        assert type(ei.value).__name__ == case["raises"]
        return
    s, z = obs.forward(x)
    assert (s, z) == (case["scale"], case["zp"]) or (math.isnan(s) and math.isnan(case["scale"]))
    assert (obs.min_val, obs.max_val) == (case["min_val"], case["max_val"])
    q = V.UniformQuantizer(case["bits"], case["sym"])
    xg = cu(G.arr(case["x"]), grad=True)
    y = q.quantize(xg, s, z, False)
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    y.backward(cu(G.arr(case["g"])))
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")
    G.assert_bitwise_f32(npy(q.discreate_tensor(x, s, z, q.qmin, q.qmax)), G.arr(case["x_int"]), "x_int")
    # sync-free device path: qparams from the observer kernel, read by pointer
    obs2 = V.MinMaxObserver(case["sym"], case["obs_bits"])
    qp, st = obs2.observe_device(x)
    qph = npy(qp)
    assert qph[H.QP_SCALE] == case["scale"] and qph[H.QP_ZP] == case["zp"]
    y2 = q.quantize(x, qp[H.QP_SCALE], qp[H.QP_ZP], False)
    G.assert_bitwise_f32(npy(y2), G.arr(case["y"]), "y(device qparams)")
    codes = FQ.fake_quant(x, s, z, q.qmin, q.qmax, want_codes=True)[2]
    xi = G.arr(case["x_int"])
    ok = ~np.isnan(xi)
    assert np.array_equal(npy(codes)[ok].astype(np.int64), xi[ok].astype(np.int64))


@pytest.mark.parametrize("case", G.cases("fixed_fq"), ids=lambda c: c["key"])
def test_golden_fixed_fq(case):
    q = V.UniformQuantizer(case["bits"], case["sym"])
    xg = cu(G.arr(case["x"]), grad=True)
    y = q.quantize(xg, case["scale"], case["zp"], False)
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    y.backward(cu(G.arr(case["g"])))
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")
    xi = q.discreate_tensor(cu(G.arr(case["x"])), case["scale"], case["zp"], q.qmin, q.qmax)
    G.assert_bitwise_f32(npy(xi), G.arr(case["x_int"]), "x_int")


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("case", G.cases("per_channel_observe_fq"), ids=lambda c: c["key"])
def test_golden_per_channel(case, fused):
    w = G.arr(case["x"])
    obs = V.PerChannelMinMaxObserver(case["sym"], case["obs_bits"])
    q = V.PerChannelUniformQuantizer(case["bits"], case["sym"])
    xg = cu(w, grad=True)
    if fused:
        y, rs = obs.observe_quantize(xg, q, want_row_stats=True)
        s, z = obs.get_scale_zero_point()
    else:
        s, z = obs.forward(xg.detach())
        y = q.quantize(xg, s, z, False)
    assert np.array_equal(npy(s), G.arr(case["scale"]), equal_nan=True)
    zg = G.arr(case["zp"]).astype(np.float64)
    assert np.array_equal(npy(z), zg)
    assert np.array_equal(npy(obs.min_val), G.arr(case["min_val"]))
    assert np.array_equal(npy(obs.max_val), G.arr(case["max_val"]))
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    y.backward(cu(G.arr(case["g"])))
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")


@pytest.mark.parametrize("case", G.cases("learnable_fq"), ids=lambda c: c["key"])
def test_golden_learnable(case):
    x, g = G.arr(case["x"]), G.arr(case["g"])
    qcls = V.UniformQuantizer if case["sym"] else V.LSQQuantizer
    q = qcls(case["bits"], case["sym"])
    scale = torch.nn.Parameter(torch.tensor(case["scale"], dtype=torch.float64, device=DEV))
    if case["sym"]:
        zp = 0
    else:
        zp = torch.nn.Parameter(torch.tensor(case["zp"], dtype=torch.float64, device=DEV))
    xg = cu(x, grad=True)
    y = q.quantize(xg, scale, zp, True)
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    y.backward(cu(g))
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")
    assert scale.grad.dtype == torch.float64
    assert float(scale.grad) == pytest.approx(case["scale_grad"], rel=1e-4, abs=1e-9)
    qmin, qmax = O.qrange(case["bits"], case["sym"])
    _, _, gs_o, gz_o = O.lsq_forward_backward(x, g, case["scale"], case["zp"], qmin, qmax,
                                              O.grad_scale(qmax, x.size), learn_zp=not case["sym"])
    assert float(scale.grad) == pytest.approx(gs_o, rel=1e-9, abs=1e-12)
    if not case["sym"]:
        assert float(zp.grad) == pytest.approx(case["zp_grad"], rel=1e-4, abs=1e-9)
        assert float(zp.grad) == pytest.approx(gz_o, rel=1e-9, abs=1e-12)


@pytest.mark.parametrize("case", G.cases("learnable_fq_calib"), ids=lambda c: c["key"])
def test_golden_learnable_calib_grad_scale_tensor(case):
    """calib_grad_scale as a per-channel device tensor (utils/estimate_bn.py:136): K4's
    gradients against the reference's (fp32 sum, <= 1e-4) and the f64 closed form."""
    x, g = G.arr(case["x"]), G.arr(case["g"])
    qcls = V.UniformQuantizer if case["sym"] else V.LSQQuantizer
    q = qcls(case["bits"], case["sym"])
    q.calib_grad_scale = cu(G.arr(case["calib"]))
    scale = torch.nn.Parameter(torch.tensor(case["scale"], dtype=torch.float64, device=DEV))
    zp = 0 if case["sym"] else torch.nn.Parameter(torch.tensor(case["zp"], dtype=torch.float64, device=DEV))
    xg = cu(x, grad=True)
    y = q.quantize(xg, scale, zp, True)
    y.backward(cu(g))
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")
    assert float(scale.grad) == pytest.approx(case["scale_grad"], rel=1e-4, abs=1e-9)
    # the factor is cached per tensor version: an in-place update is picked up
    q.calib_grad_scale.mul_(2.0)
    xg.grad = None
    scale.grad = None
    q.quantize(xg, scale, zp, True).backward(cu(g))
    assert float(scale.grad) == pytest.approx(2 * case["scale_grad"], rel=1e-4, abs=1e-9)
    q.calib_grad_scale.mul_(0.5)
    scale.grad = None
    if not case["sym"]:
        zp.grad = None
    q.quantize(xg, scale, zp, True).backward(cu(g))
    qmin, qmax = O.qrange(case["bits"], case["sym"])
    calib = float(G.arr(case["calib"]).astype(np.float64).sum())   # sum_to of ScaleGradient's grad
    _, _, gs_o, gz_o = O.lsq_forward_backward(x, g, case["scale"], case["zp"], qmin, qmax,
                                              O.grad_scale(qmax, x.size, calib), learn_zp=not case["sym"])
    assert float(scale.grad) == pytest.approx(gs_o, rel=1e-9, abs=1e-12)
    if not case["sym"]:
        assert float(zp.grad) == pytest.approx(case["zp_grad"], rel=1e-4, abs=1e-9)
        assert float(zp.grad) == pytest.approx(gz_o, rel=1e-9, abs=1e-12)


def test_asym_learnable_int_zero_point_raises_like_reference():
    q = V.UniformQuantizer(8, False)
    s = torch.nn.Parameter(torch.tensor(0.1, dtype=torch.float64, device=DEV))
    with pytest.raises(TypeError):
        q.quantize(torch.randn(10, device=DEV), s, 0, True)


@pytest.mark.parametrize("mode", ["reference", "default"])
@pytest.mark.parametrize("case", G.cases("manager_sequence"), ids=lambda c: c["key"])
def test_golden_manager_sequence(case, mode):
    """calibrate (observe only) -> observe+quantize -> init_scaling_factor_for_learning ->
    make_learn_qparameter -> one learnable step, nothing injected.  "reference": mean|x| /
    mean x as torch's CPU kernel sums them on the golden host (H.set_mean_reference, K11),
    so the learnable scale and the step are the reference's bit for bit.  "default" (no
    extra pass): the means are the correctly rounded fp32 ones, within 1e-6; the scale's
    fp32 value may then differ by an ulp, so y equals the reference's in its integer
    codes, not in every bit."""
    if mode == "reference":
        H.set_mean_reference(G.GOLDEN_SILU_REF[1])
    try:
        _manager_sequence(case, exact=mode == "reference")
    finally:
        H.clear_mean_reference()


def _manager_sequence(case, exact):
    qm = V.QuantizationManager("UniformQuantizer", "MinMaxObserver", case["bits"], case["sym"], True)
    qm.is_observer_qparam, qm.is_learning_scale, qm.is_quantize = True, False, False
    outs = [(qm.quantize(cu(G.arr(k))), k) for k in case["xs"]]
    assert all(np.array_equal(npy(o), G.arr(k)) for o, k in outs)
    cal = case["calib"]
    assert (qm.observer.min_val, qm.observer.max_val) == (cal["min_val"], cal["max_val"])
    assert float(qm.scale) == cal["scale"] and float(qm.zero_point) == cal["zero_point"]
    if exact:
        assert [float(v) for v in qm.mean_abs_x] == cal["mean_abs_x"]
        assert [float(v) for v in qm.mean_x] == cal["mean_x"]
        assert [float(v) for v in qm.std] == cal["std"]
    else:
        np.testing.assert_allclose(qm.mean_abs_x, cal["mean_abs_x"], rtol=1e-6)
        np.testing.assert_allclose(qm.mean_x, cal["mean_x"], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(qm.std, cal["std"], rtol=1e-6)
    # every recorded value is an fp32 value, as the reference's .item() of an fp32 tensor
    for v in list(qm.mean_abs_x) + list(qm.mean_x) + list(qm.std):
        assert float(np.float32(v)) == v
    qm.is_quantize = True
    y = qm.quantize(cu(G.arr(case["x_oq"])))
    G.assert_bitwise_f32(npy(y), G.arr(case["y_oq"]), "observe+quantize")
    qm.is_learning_scale = True
    qm.init_scaling_factor_for_learning()
    if exact:
        assert qm.scale == case["init_scale"]
    else:
        assert qm.scale == pytest.approx(case["init_scale"], rel=1e-6)
    qm.make_learn_qparameter()
    assert isinstance(qm.scale, torch.nn.Parameter) and qm.scale.dtype == torch.float64
    if "learn_raises" in case:
        with pytest.raises(TypeError):
            qm.quantize(cu(G.arr(case["xs"][0])))
        return
    qm.cuda()
    xg = cu(G.arr(case["x4"]), grad=True)
    y4 = qm.quantize(xg)
    if exact:
        G.assert_bitwise_f32(npy(y4), G.arr(case["y4"]), "y4")
    else:   # the same integer codes under each side's own fp32 scale
        s_ours, s_ref = np.float32(float(qm.scale)), np.float32(case["init_scale"])
        np.testing.assert_array_equal(np.rint(npy(y4) / s_ours), np.rint(G.arr(case["y4"]) / s_ref))
    y4.backward(cu(G.arr(case["g4"])))
    if exact:
        G.assert_bitwise_f32(npy(xg.grad), G.arr(case["gx4"]), "gx4")
    else:
        np.testing.assert_array_equal(npy(xg.grad) != 0, G.arr(case["gx4"]) != 0)
    assert float(qm.scale.grad) == pytest.approx(case["scale_grad"], rel=1e-4)


# --------------------------------------------------------------------------- oracle, seeded
def _rand(shape, seed, scale=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * scale).astype(np.float32)


@pytest.mark.parametrize("shape", [(1024, 1024, 3, 3), (16, 3, 3, 3), (64, 7, 5, 5), (3, 20000),
                                   (256, 40), (5, 4, 1, 1)])
@pytest.mark.parametrize("sym,bits", [(False, 8), (True, 8), (True, 4), (False, 2)])
def test_per_channel_vs_oracle(shape, sym, bits):
    """C2 (north-star shape) and odd shapes: vector / scalar / large-row kernels."""
    w = _rand(shape, 7, 0.05)
    q = V.PerChannelUniformQuantizer(bits, sym)
    obs = V.PerChannelMinMaxObserver(sym)
    y, _ = obs.observe_quantize(cu(w), q)
    s, z = obs.get_scale_zero_point()
    ref = O.per_channel_observe_fq(w, sym, bits, 8)
    assert np.array_equal(npy(s), ref["scale"])
    assert np.array_equal(npy(z), ref["zp"].astype(np.float64))
    G.assert_bitwise_f32(npy(y), ref["y"], "y")
    codes = FQ.per_channel_observe_fq(cu(w), symmetric=sym, qmin=q.qmin, qmax=q.qmax,
                                      want_codes=True, want_mask=True)
    assert np.array_equal(npy(codes["codes"]).astype(np.int64), ref["x_int"].astype(np.int64))
    C = shape[0]
    m = G.unpack_mask(npy(codes["mask"]), C, w.size // C)
    assert np.array_equal(m, ref["mask"].reshape(C, -1))


def test_per_channel_fwd_bwd_c2_full():
    """North-star step at full size: per-channel asym int8 observe+fq fwd + STE bwd."""
    w = _rand((1024, 1024, 3, 3), 0, 0.05)
    g = _rand((1024, 1024, 3, 3), 1)
    q = V.PerChannelUniformQuantizer(8, False)
    obs = V.PerChannelMinMaxObserver(False)
    xg = cu(w, grad=True)
    y, _ = obs.observe_quantize(xg, q)
    y.backward(cu(g))
    ref = O.per_channel_observe_fq(w, False, 8, 8)
    G.assert_bitwise_f32(npy(y), ref["y"], "y")
    G.assert_bitwise_f32(npy(xg.grad), O.per_channel_backward_fixed(g, ref["mask"], ref["scale"]), "gx")


def test_per_channel_running_state_and_nan_rows():
    """Two calls on one observer: running min/max per channel, NaN row leaves its state."""
    w1 = _rand((6, 50), 3)
    w2 = _rand((6, 50), 4) * 3
    w2[2, 5] = np.nan
    obs = V.PerChannelMinMaxObserver(False)
    q = V.PerChannelUniformQuantizer(8, False)
    obs.observe_quantize(cu(w1), q)
    y2, _ = obs.observe_quantize(cu(w2), q)
    r1 = O.per_channel_observe_fq(w1, False, 8, 8)
    ref = O.per_channel_observe_fq(w2, False, 8, 8, run_min=r1["min_val"], run_max=r1["max_val"])
    assert np.array_equal(npy(obs.min_val), ref["min_val"])
    assert np.array_equal(npy(obs.max_val), ref["max_val"])
    assert ref["min_val"][2] == r1["min_val"][2] and ref["max_val"][2] == r1["max_val"][2]
    G.assert_bitwise_f32(npy(y2), ref["y"], "y2")


@pytest.mark.parametrize("n", [1, 3, 4, 1023, 4097, 1 << 20, (1 << 20) + 5])
@pytest.mark.parametrize("sym", [True, False])
def test_per_tensor_observe_fq_sizes(n, sym):
    x = _rand(n, n % 97, 2.0)
    obs = V.MinMaxObserver(sym)
    qp, st = obs.observe_device(cu(x))
    mn, mx = O.observe_minmax(x, 0, 0)
    s, z = O.minmax_qparams(mn, mx, sym, 8)
    qph = npy(qp)
    assert qph[H.QP_SCALE] == s and qph[H.QP_ZP] == z
    sth = npy(st)
    ma, me, sd = O.collect_stats(x)
    assert sth[H.ST_MEANABS] == pytest.approx(ma, rel=1e-6)
    if n > 1:
        assert sth[H.ST_STD] == pytest.approx(sd, rel=1e-6)
    q = V.UniformQuantizer(4, sym)
    y = q.quantize(cu(x), qp[H.QP_SCALE], qp[H.QP_ZP], False)
    yo, _, _ = O.fq_forward(x, s, z, q.qmin, q.qmax)
    G.assert_bitwise_f32(npy(y), yo, "y")


def test_misaligned_and_noncontiguous_inputs():
    base = _rand(4099, 11)
    xt = cu(base)[3:]                        # 12-byte offset: scalar kernel path
    q = V.UniformQuantizer(8, True)
    y = q.quantize(xt, 0.02, 0, False)
    G.assert_bitwise_f32(npy(y), O.fq_forward(base[3:], 0.02, 0, -128, 127)[0], "misaligned")
    m = _rand((64, 48), 12)
    y2 = q.quantize(cu(m).t(), 0.02, 0, False)  # non-contiguous -> contiguous copy
    G.assert_bitwise_f32(npy(y2), O.fq_forward(m.T.copy(), 0.02, 0, -128, 127)[0], "transposed")


def test_empty_tensor():
    q = V.UniformQuantizer(8, True)
    assert q.quantize(torch.empty(0, device=DEV), 0.1, 0, False).numel() == 0
    with pytest.raises(RuntimeError):
        V.MinMaxObserver(True).forward(torch.empty(0, device=DEV))


@pytest.mark.parametrize("sym", [True, False])
def test_lsq_c3_full_size(sym):
    """C3: 512x3x224x224 learnable fwd + STE bwd; grad_x bitwise, scale grad vs f64 closed form."""
    shape = (512, 3, 224, 224)
    x = _rand(shape, 0)
    g = _rand(shape, 1)
    qcls = V.UniformQuantizer if sym else V.LSQQuantizer
    q = qcls(8, sym)
    scale = torch.nn.Parameter(torch.tensor(0.03, dtype=torch.float64, device=DEV))
    zp = 0 if sym else torch.nn.Parameter(torch.tensor(3.0, dtype=torch.float64, device=DEV))
    xg = cu(x, grad=True)
    y = q.quantize(xg, scale, zp, True)
    y.backward(cu(g))
    qmin, qmax = O.qrange(8, sym)
    yo, gxo, gso, gzo = O.lsq_forward_backward(x, g, 0.03, 0 if sym else 3.0, qmin, qmax,
                                               O.grad_scale(qmax, x.size), learn_zp=not sym)
    G.assert_bitwise_f32(npy(y), yo, "y")
    G.assert_bitwise_f32(npy(xg.grad), gxo, "grad_x")
    assert float(scale.grad) == pytest.approx(gso, rel=1e-9)
    if not sym:
        assert float(zp.grad) == pytest.approx(gzo, rel=1e-9)


@pytest.mark.parametrize("groups", [0, 2, 4, 8, 16])
@pytest.mark.parametrize("n", [1, 4099, 295_000, 525_000, 3_276_800, 13_107_200, 21_000_003])
def test_lsq_groups_per_lane_sizes(n, groups):
    """K4 at 2 / 4 / 8 / 16 groups per lane (VSIQ_TUNE_LSQ_GROUPS; 0 = default: 4, 8 from
    20M elements), grids from 1
    to >12k workgroups (flat and two-level partial folds): grad_x bitwise, f64 scale
    gradient vs the oracle's closed form."""
    x = _rand(n, n % 97, 0.5)
    g = _rand(n, n % 89 + 1)
    H.set_tuning(H.TUNE_LSQ_GROUPS, groups)
    try:
        gx, grads = FQ.lsq_backward(cu(g), cu(x), 0.01, 0, -8, 7, 0.37, False)
    finally:
        H.set_tuning(H.TUNE_LSQ_GROUPS, 0)
    _, gxo, gso, _ = O.lsq_forward_backward(x, g, 0.01, 0, -8, 7, 0.37)
    G.assert_bitwise_f32(npy(gx), gxo, "grad_x")
    assert float(grads[0]) == pytest.approx(gso, rel=1e-9, abs=1e-12)


@pytest.mark.parametrize("obs_kernel", [1, 2])
@pytest.mark.parametrize("n", [1, 4099, 525_000, 3_276_800, 13_107_200, 21_000_003])
def test_observer_kernels_sizes(n, obs_kernel):
    """K2 one-shot (flat and two-level folds) and grid-stride forms against the oracle."""
    x = _rand(n, n % 61 + 3, 0.7)
    H.set_tuning(H.TUNE_OBS_KERNEL, obs_kernel)
    try:
        side = torch.cuda.Stream()   # a fresh (device, stream) workspace sized for this n only
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            qp, st = FQ.observe_tensor(cu(x), symmetric=False)
        torch.cuda.current_stream().wait_stream(side)
    finally:
        H.set_tuning(H.TUNE_OBS_KERNEL, 0)
    mn, mx = O.observe_minmax(x)
    st = npy(st)
    assert (st[H.ST_MIN], st[H.ST_MAX]) == (float(x.min()), float(x.max()))
    x64 = x.astype(np.float64)   # sums: f64 over fp32 partials of 4 elements (<= 1e-6)
    assert st[H.ST_SUMABS] == pytest.approx(np.abs(x64).sum(), rel=1e-6)
    assert st[H.ST_SUM] == pytest.approx(x64.sum(), rel=1e-6, abs=1e-6 * np.abs(x64).sum())
    assert st[H.ST_SUMSQ] == pytest.approx((x64 * x64).sum(), rel=1e-6)
    scale, zp = O.minmax_qparams(mn, mx, False)
    q = npy(qp)
    assert (q[H.QP_SCALE], q[H.QP_ZP]) == (scale, zp)


def test_reductions_deterministic():
    x = cu(_rand(3_000_001, 5))
    g = cu(_rand(3_000_001, 6))
    outs = []
    for _ in range(3):
        _, st = FQ.observe_tensor(x, symmetric=True)
        _, grads = FQ.lsq_backward(g, x, 0.05, 0, -128, 127, 1e-3, False)
        outs.append((npy(st).tobytes(), npy(grads).tobytes()))
    assert outs[0] == outs[1] == outs[2]


def test_fast_division_exhaustive():
    """The kernels' reciprocal + Newton-Markstein division equals IEEE x/s for ALL 2^32 x."""
    rng = np.random.default_rng(3)
    divs = [1.0, 3.0, 0.1, 0.03, 1.9999999, 1.0000001, 2.0 ** -60, 2.0 ** 60, 7.0e-3,
            np.float32(np.nextafter(np.float32(2), np.float32(0))), 255.00001, 0.0, -0.5,
            float("inf"), 1e-30, 3.4e38] + list(rng.uniform(1e-4, 10.0, 8))
    b = torch.tensor(np.asarray(divs, np.float32), device=DEV)
    bad = torch.zeros(len(divs), dtype=torch.int64, device=DEV)
    H.check(H.lib().vsiq_selftest_div(H.ptr(b), len(divs), H.ptr(bad), H.stream_of(b.device)),
            "vsiq_selftest_div")
    assert npy(bad).tolist() == [0] * len(divs)


def _selftest_fq(mode, scales, zps, lo, hi):
    s = torch.tensor(np.asarray(scales, np.float32), device=DEV)
    z = torch.tensor(np.asarray(zps, np.float32), device=DEV)
    out = torch.zeros(2 * len(scales), dtype=torch.int64, device=DEV)
    H.check(H.lib().vsiq_selftest_fq(mode, H.ptr(s), H.ptr(z), len(scales), float(lo), float(hi),
                                     H.ptr(out), H.stream_of(s.device)), "vsiq_selftest_fq")
    return npy(out).reshape(-1, 2)


def test_fast_quantizer_exhaustive():
    """The no-check forward element (fq_elem_fast) gives the reference's code c =
    clamp(rint(x/s + zp)) -- value, sign of zero and STE mask bit -- for ALL 2^32 x
    with |x| <= 2^62, for scales/zero points inside the fast domain; outside it the
    kernels take the IEEE path (checked count 0 here)."""
    ones = float(np.float32(np.nextafter(np.float32(2), np.float32(0))))
    pairs = [(2.0 ** -20, 0.0), (2.0 ** 62, 0.0), (0.0123, 0.0), (1 / 127, 0.0), (ones, 0.0),
             (0.05, 3.0), (0.02, -5.0), (0.1, 128.0), (3.7, 0.37), (0.3, 2.0 ** -12),
             (1e-3, -2.5), (2.0 ** -19 * 1.7, 1.0), (1e5, 0.0), (0.031, 255.0), (1.0, 0.5),
             (2.0 ** -21, 0.0), (0.1, 1e-5), (0.1, float("nan"))]      # last three: outside
    for lo, hi in ((-128, 127), (0, 255), (-2, 1)):
        res = _selftest_fq(0, [p[0] for p in pairs], [p[1] for p in pairs], lo, hi)
        assert res[:, 0].tolist() == [0] * len(pairs), (lo, hi, res.tolist())
        assert (res[:-3, 1] > 3_100_000_000).all() and (res[-3:, 1] == 0).all(), res.tolist()


def test_fast_ste_division_exhaustive():
    """ste_quot(g) = RN(RN(g*s)/s) for ALL 2^32 g inside its domain."""
    rng = np.random.default_rng(5)
    ones = float(np.float32(np.nextafter(np.float32(2), np.float32(0))))
    scales = [2.0 ** -60, 2.0 ** 60, 0.1, 1 / 3, ones, 1.0, 0.0123, 1 / 127, 255.00001,
              float(np.float32(np.nextafter(np.float32(1), np.float32(0)))), 2.0 ** -61] + \
        list(rng.uniform(1e-4, 10.0, 6))
    res = _selftest_fq(1, scales, [0.0] * len(scales), 0, 0)
    assert res[:, 0].tolist() == [0] * len(scales), res.tolist()
    assert (np.delete(res[:, 1], 10) > 1_700_000_000).all() and res[10, 1] == 0, res.tolist()


def test_tail_groups_and_mask_bits_per_tensor():
    """n % 4 != 0 and n % 256 != 0: scalar groups, partial ballots."""
    for n in (5, 255, 257, 1001, 4099):
        x = _rand(n, n, 3.0)
        g = _rand(n, n + 1)
        q = V.UniformQuantizer(4, False)
        y, mask, codes = FQ.fake_quant(cu(x), 0.4, 3, q.qmin, q.qmax, want_mask=True, want_codes=True)
        yo, qo, mo = O.fq_forward(x, 0.4, 3, q.qmin, q.qmax)
        G.assert_bitwise_f32(npy(y), yo, "y")
        assert np.array_equal(G.unpack_mask(npy(mask), 1, n)[0], mo)
        assert np.array_equal(npy(codes).astype(np.int64), qo.astype(np.int64))
        gx = FQ.ste_backward(cu(g), mask, 0.4)
        G.assert_bitwise_f32(npy(gx), O.fq_backward_fixed(g, mo, 0.4), "gx")


def test_cpu_tensor_takes_the_host_path():
    """A CPU tensor is computed by the native host loops (vsiquantization_amd/host.py),
    stays on the CPU and equals the oracle; a CUDA op handed a CPU operand still raises."""
    x = np.random.default_rng(3).standard_normal(1000).astype(np.float32)
    y = V.UniformQuantizer(8, True).quantize(torch.from_numpy(x), 0.1, 0, False)
    assert y.device.type == "cpu"
    G.assert_bitwise_f32(y.numpy(), O.fq_forward(x, 0.1, 0, -128, 127)[0], "host y")
    g = torch.randn(64, device=DEV)
    _, mask, _ = FQ.fake_quant(g, 0.1, 0, -128, 127, want_mask=True)
    with pytest.raises(H.VsiqError):
        FQ.ste_backward(g, mask, 0.1, pre=torch.randn(64), act="relu")


@pytest.mark.parametrize("case", G.cases("learnable_fq_sym_tensor_zp"), ids=lambda c: c["key"])
def test_golden_learnable_sym_tensor_zp(case):
    """Symmetric learnable quantize with a gradient-requiring tensor zero point on the GPU
    (K1 with zp as given + K4 zp_learn 2): y / grad_x bitwise vs the reference, the scale
    and zero-point gradients to its fp32 sums (1e-4) and the oracle's f64 form (1e-9)."""
    x, g = G.arr(case["x"]), G.arr(case["g"])
    q = V.UniformQuantizer(case["bits"], True)
    scale = torch.nn.Parameter(torch.tensor(case["scale"], dtype=torch.float64, device=DEV))
    zp = torch.nn.Parameter(torch.tensor(case["zp"], dtype=torch.float64, device=DEV))
    xg = cu(x, grad=True)
    y = q.quantize(xg, scale, zp, True)
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    y.backward(cu(g))
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")
    # the reference sums ~3K fp32 terms in fp32 (error ~1e-6 absolute; these gradients
    # cancel down to 1e-3..1e-2): 1e-4 relative or 3e-6 absolute; the oracle's f64 closed
    # form below is the tight check
    assert float(scale.grad) == pytest.approx(case["scale_grad"], rel=1e-4, abs=3e-6)
    assert float(zp.grad) == pytest.approx(case["zp_grad"], rel=1e-4, abs=3e-6)
    qmin, qmax = O.qrange(case["bits"], True)
    _, _, gs_o, gz_o = O.lsq_forward_backward(x, g, case["scale"], case["zp"], qmin, qmax,
                                              O.grad_scale(qmax, x.size), learn_zp=2)
    assert float(scale.grad) == pytest.approx(gs_o, rel=1e-9, abs=1e-12)
    assert float(zp.grad) == pytest.approx(gz_o, rel=1e-9, abs=1e-12)


@pytest.mark.parametrize("case", G.cases("per_channel_learnable"), ids=lambda c: c["key"])
def test_golden_per_channel_learnable(case):
    """Learnable PerChannelUniformQuantizer (K3-fixed forward, K6 backward on axis 0) ==
    the reference's learnable UniformQuantizer per out-channel row."""
    w, g = G.arr(case["x"]), G.arr(case["g"])
    sym, bits = case["sym"], case["bits"]
    q = V.PerChannelUniformQuantizer(bits, sym)
    s0, z0 = G.arr(case["scale"]), G.arr(case["zp"])
    scale = torch.nn.Parameter(cu(s0.copy()))
    zp = 0 if sym else torch.nn.Parameter(cu(z0.copy()))
    xg = cu(w, grad=True)
    y = q.quantize(xg, scale, zp, True)
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    y.backward(cu(g))
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")
    np.testing.assert_allclose(npy(scale.grad), G.arr(case["scale_grad"]), rtol=1e-4, atol=3e-6)
    if not sym:
        np.testing.assert_allclose(npy(zp.grad), G.arr(case["zp_grad"]), rtol=1e-4, atol=3e-6)


@pytest.mark.parametrize("act", [None, "relu"])
def test_nontemporal_off_equals_default(act):
    """VSIQ_TUNE_NONTEMPORAL 0 (cached loads / stores in every streamed kernel, the knob an
    operator A/B-tests on a box) gives the default's bits: K3 per-channel observe + fake
    quant and its STE backward, K2 + K1 per tensor, K4, K2o deferred records."""
    g0 = torch.Generator(device=DEV).manual_seed(31)
    w = torch.randn(256, 64, 3, 3, device=DEV, generator=g0) * 0.05
    x = torch.randn(8, 32, 40, 40, device=DEV, generator=g0)
    gy = torch.randn(8, 32, 40, 40, device=DEV, generator=g0)

    def run():
        out = []
        r = FQ.per_channel_observe_fq(w, symmetric=False, qmin=0, qmax=255, want_mask=True)
        out += [r["y"], r["scale"], r["zp"]]
        qp, st = FQ.observe_tensor(x, symmetric=True, act=act)
        y, mask, _ = FQ.fake_quant(x, None, None, -128, 127, qp=qp, want_mask=True, act=act)
        out += [qp, st, y, FQ.ste_backward(gy, mask, qp[H.QP_SCALE:H.QP_SCALE + 1], pre=x if act else None,
                                            act=act)]
        gx, grads = FQ.lsq_backward(gy, x, 0.02, 3.0, -8, 7, 0.37, True, act=act)
        out += [gx, grads]
        yo, slot = FQ.observe_parts_out(x, act or "relu")
        out += [yo, FQ.fold_parts(slot.reshape(1, -1))]
        torch.cuda.synchronize()
        return [o.detach().clone() for o in out]

    base = run()
    H.set_tuning(H.TUNE_NONTEMPORAL, 0)
    try:
        off = run()
    finally:
        H.set_tuning(H.TUNE_NONTEMPORAL, 1)
    for i, (a, b) in enumerate(zip(base, off)):
        a, b = a.reshape(-1), b.reshape(-1)
        if a.dtype == torch.float64:
            assert torch.equal(a.view(torch.int64), b.view(torch.int64)) or torch.allclose(a, b, rtol=1e-15), i
        else:
            assert torch.equal(a.view(torch.int32), b.view(torch.int32)), i
