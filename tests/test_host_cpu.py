"""The native host path (CPU tensors; csrc/k_host.hip through vsiquantization_amd/host.py)
against the reference goldens, bit for bit: the reference's own environment
(BASELINE C1: UniformQuantizer / MinMaxObserver on CPU tensors).  Runs without a GPU."""
import math

import numpy as np
import pytest
import torch

import vsiquantization_amd as V
from vsiquantization_amd import _hip as H
from vsiquantization_amd import host
from oracle import fakequant_np as O
from tests import goldens as G


def t(a, grad=False):
    x = torch.from_numpy(np.ascontiguousarray(a))
    return x.requires_grad_(True) if grad else x


def npy(x):
    return x.detach().numpy()


@pytest.mark.parametrize("case", G.cases("per_tensor_observe_fq"), ids=lambda c: c["key"])
def test_golden_per_tensor_observe_fq(case):
    x = t(G.arr(case["x"]))
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
    xg = t(G.arr(case["x"]), grad=True)
    y = q.quantize(xg, s, z, False)
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    y.backward(t(G.arr(case["g"])))
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")
    G.assert_bitwise_f32(npy(q.discreate_tensor(x, s, z, q.qmin, q.qmax)), G.arr(case["x_int"]), "x_int")
    # the qparams record of the host pass, read as a tensor
    obs2 = V.MinMaxObserver(case["sym"], case["obs_bits"])
    qp, _ = obs2.observe_device(x)
    assert qp[H.QP_SCALE].item() == case["scale"] and qp[H.QP_ZP].item() == case["zp"]
    G.assert_bitwise_f32(npy(q.quantize(x, qp[H.QP_SCALE], qp[H.QP_ZP], False)), G.arr(case["y"]), "y(record)")


@pytest.mark.parametrize("case", G.cases("fixed_fq"), ids=lambda c: c["key"])
def test_golden_fixed_fq(case):
    q = V.UniformQuantizer(case["bits"], case["sym"])
    xg = t(G.arr(case["x"]), grad=True)
    y = q.quantize(xg, case["scale"], case["zp"], False)
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    y.backward(t(G.arr(case["g"])))
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")


@pytest.mark.parametrize("case", G.cases("learnable_fq"), ids=lambda c: c["key"])
def test_golden_learnable(case):
    x, g = G.arr(case["x"]), G.arr(case["g"])
    q = (V.UniformQuantizer if case["sym"] else V.LSQQuantizer)(case["bits"], case["sym"])
    scale = torch.nn.Parameter(torch.tensor(case["scale"], dtype=torch.float64))
    zp = 0 if case["sym"] else torch.nn.Parameter(torch.tensor(case["zp"], dtype=torch.float64))
    xg = t(x, grad=True)
    y = q.quantize(xg, scale, zp, True)
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    y.backward(t(g))
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")
    assert float(scale.grad) == pytest.approx(case["scale_grad"], rel=1e-4, abs=1e-9)
    qmin, qmax = O.qrange(case["bits"], case["sym"])
    _, _, gs_o, gz_o = O.lsq_forward_backward(x, g, case["scale"], case["zp"], qmin, qmax,
                                              O.grad_scale(qmax, x.size), learn_zp=not case["sym"])
    assert float(scale.grad) == pytest.approx(gs_o, rel=1e-9, abs=1e-12)
    if not case["sym"]:
        assert float(zp.grad) == pytest.approx(case["zp_grad"], rel=1e-4, abs=1e-9)


@pytest.mark.parametrize("case", G.cases("manager_sequence"), ids=lambda c: c["key"])
def test_golden_manager_sequence(case):
    """QuantizationManager on CPU tensors: calibrate (stats lists, running min/max,
    qparams), observe + quantize, learn-init (qm.py:55-114)."""
    bits, sym = case["bits"], case["sym"]
    qm = V.QuantizationManager("UniformQuantizer", "MinMaxObserver", bits, sym, is_learning_scale=False)
    qm.is_observer_qparam, qm.is_quantize = True, False
    for k in case["xs"]:
        qm.quantize(t(G.arr(k)))
    cal = case["calib"]
    assert (qm.observer.min_val, qm.observer.max_val) == (cal["min_val"], cal["max_val"])
    assert (qm.scale, qm.zero_point) == (cal["scale"], cal["zero_point"])
    np.testing.assert_allclose(qm.mean_abs_x, cal["mean_abs_x"], rtol=1e-6)
    np.testing.assert_allclose(qm.mean_x, cal["mean_x"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(qm.std, cal["std"], rtol=1e-6)
    qm.is_quantize = True
    y = qm.quantize(t(G.arr(case["x_oq"])))
    assert qm.scale == case["observe_quantize"]["scale"]
    G.assert_bitwise_f32(npy(y), G.arr(case["y_oq"]), "y_oq")


@pytest.mark.parametrize("case", G.cases("act_fq"), ids=lambda c: c["key"])
def test_golden_act_fq(case):
    """Fused ReLU / SiLU + fake quant on the host (torch CPU's SiLU bits, this layout)."""
    H.set_silu_reference(*G.GOLDEN_SILU_REF)
    try:
        q = V.UniformQuantizer(case["bits"], case["sym"])
        c = t(G.arr(case["x"]), grad=True)
        if case["mode"] == "observe":
            qp, _ = host.observe_tensor(c.detach(), symmetric=case["sym"], act=case["act"])
            assert (qp[H.QP_SCALE].item(), qp[H.QP_ZP].item()) == (case["scale"], case["zp"])
            y = host.fake_quant_fixed(c, None, None, q.qmin, q.qmax, qp=qp, act=case["act"])
        elif case["mode"] == "fixed":
            y = q.quantize(c, case["scale"], case["zp"], False, act=case["act"])
        else:
            s = torch.nn.Parameter(torch.tensor(case["scale"], dtype=torch.float64))
            y = q.quantize(c, s, 0, True, act=case["act"])
        y.backward(t(G.arr(case["g"])))
        G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
        G.assert_bitwise_f32(npy(c.grad), G.arr(case["grad_x"]), "grad_c")
    finally:
        H.set_silu_reference()


def test_c1_full_size_vs_oracle():
    """BASELINE C1 (256x256 per-tensor symmetric int8) through the public classes on the
    host, against the oracle: qparams exact, y / codes / grad bitwise."""
    rng = np.random.default_rng(1)
    w = (rng.standard_normal((256, 256)) * 0.05).astype(np.float32)
    g = rng.standard_normal((256, 256)).astype(np.float32)
    obs, q = V.MinMaxObserver(True), V.UniformQuantizer(8, True)
    s, z = obs.forward(t(w))
    mn, mx = O.observe_minmax(w)
    assert (s, z) == O.minmax_qparams(mn, mx, True, 8)
    xg = t(w, grad=True)
    y = q.quantize(xg, s, z, False)
    y.backward(t(g))
    yo, qo, mo = O.fq_forward(w, s, z, -128, 127)
    G.assert_bitwise_f32(npy(y), yo, "y")
    G.assert_bitwise_f32(npy(xg.grad), O.fq_backward_fixed(g, mo, s), "grad")


@pytest.mark.parametrize("n", [1, 5, 65_536 * 3 + 7])
def test_host_stats_record_vs_oracle(n):
    """mean|x| / mean / std of the host pass (f64 sums in fixed chunk order) vs the oracle;
    min / max / NaN exact; a NaN call leaves the running state alone."""
    rng = np.random.default_rng(n)
    x = (rng.standard_normal(n) * 2).astype(np.float32)
    run = torch.zeros(2)
    qp, st = host.observe_tensor(t(x), symmetric=False, run_minmax=run)
    mn, mx = O.observe_minmax(x)
    assert (st[H.ST_MIN].item(), st[H.ST_MAX].item()) == (float(x.min()), float(x.max()))
    assert (run[0].item(), run[1].item()) == (mn, mx)
    ma, me, sd = O.collect_stats(x)
    assert st[H.ST_MEANABS].item() == pytest.approx(ma, rel=1e-6)
    if n > 1:
        assert st[H.ST_STD].item() == pytest.approx(sd, rel=1e-6)
    x[0] = np.nan
    run2 = run.clone()
    host.observe_tensor(t(x * 3), symmetric=False, run_minmax=run2)
    assert torch.equal(run, run2)


def test_host_threads_reported():
    assert host.threads() >= 1


@pytest.mark.parametrize("case", G.cases("learnable_fq_sym_tensor_zp"), ids=lambda c: c["key"])
def test_golden_learnable_sym_tensor_zp(case):
    """UniformQuantizer(bits, True).quantize(x, scale, zp_tensor_requiring_grad, True) on
    CPU tensors (host path, zp_learn 2) == the reference: y / grad_x bitwise, gradients
    to the reference's fp32 sums (1e-4) and the oracle's f64 closed form (1e-9)."""
    x, g = G.arr(case["x"]), G.arr(case["g"])
    q = V.UniformQuantizer(case["bits"], True)
    scale = torch.nn.Parameter(torch.tensor(case["scale"], dtype=torch.float64))
    zp = torch.nn.Parameter(torch.tensor(case["zp"], dtype=torch.float64))
    xg = t(x, grad=True)
    y = q.quantize(xg, scale, zp, True)
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    y.backward(t(g))
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


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("case", G.cases("per_channel_observe_fq"), ids=lambda c: c["key"])
def test_golden_per_channel_on_cpu(case, fused):
    """PerChannelMinMaxObserver / PerChannelUniformQuantizer on CPU tensors (the native host
    loops row by row) == the reference classes looped over out-channels."""
    w = G.arr(case["x"])
    obs = V.PerChannelMinMaxObserver(case["sym"], case["obs_bits"])
    q = V.PerChannelUniformQuantizer(case["bits"], case["sym"])
    xg = t(w, grad=True)
    if fused:
        y, rs = obs.observe_quantize(xg, q, want_row_stats=True)
        s, z = obs.get_scale_zero_point()
        assert rs.shape == (w.shape[0], 3)
    else:
        s, z = obs.forward(xg.detach())
        y = q.quantize(xg, s, z, False)
    assert s.device.type == "cpu" and z.device.type == "cpu"
    assert np.array_equal(npy(s), G.arr(case["scale"]), equal_nan=True)
    assert np.array_equal(npy(z), G.arr(case["zp"]).astype(np.float64))
    assert np.array_equal(npy(obs.min_val), G.arr(case["min_val"]))
    assert np.array_equal(npy(obs.max_val), G.arr(case["max_val"]))
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    y.backward(t(G.arr(case["g"])))
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")


@pytest.mark.parametrize("case", G.cases("per_channel_learnable"), ids=lambda c: c["key"])
def test_golden_per_channel_learnable_on_cpu(case):
    """Learnable PerChannelUniformQuantizer on CPU tensors == the reference's learnable
    UniformQuantizer.quantize per out-channel row: y / grad_x bitwise, per-row scale and
    zero-point gradients to the reference's fp32 sums (1e-4) and the f64 closed form."""
    w, g = G.arr(case["x"]), G.arr(case["g"])
    sym, bits = case["sym"], case["bits"]
    q = V.PerChannelUniformQuantizer(bits, sym)
    s0, z0 = G.arr(case["scale"]), G.arr(case["zp"])
    scale = torch.nn.Parameter(torch.from_numpy(s0.copy()))
    zp = 0 if sym else torch.nn.Parameter(torch.from_numpy(z0.copy()))
    xg = t(w, grad=True)
    y = q.quantize(xg, scale, zp, True)
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    y.backward(t(g))
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")
    np.testing.assert_allclose(npy(scale.grad), G.arr(case["scale_grad"]), rtol=1e-4, atol=3e-6)
    qmin, qmax = O.qrange(bits, sym)
    C = w.shape[0]
    for c in range(C):
        _, _, gs_o, gz_o = O.lsq_forward_backward(w[c], g[c], s0[c], z0[c], qmin, qmax,
                                                  O.grad_scale(qmax, w[c].size), learn_zp=not sym)
        assert float(scale.grad[c]) == pytest.approx(gs_o, rel=1e-9, abs=1e-12)
        if not sym:
            assert float(zp.grad[c]) == pytest.approx(gz_o, rel=1e-9, abs=1e-12)
    if not sym:
        np.testing.assert_allclose(npy(zp.grad), G.arr(case["zp_grad"]), rtol=1e-4, atol=3e-6)


def test_per_channel_host_rows_parallel_equal_single_rows():
    """Many rows (the pool over rows) and a few long rows (the pool inside each row) give
    each row exactly what the per-tensor host path gives that row alone."""
    rng = np.random.default_rng(3)
    for shape in ((64, 3, 3, 3), (3, 70000)):
        w = (rng.standard_normal(shape) * 0.1).astype(np.float32)
        obs = V.PerChannelMinMaxObserver(False)
        q = V.PerChannelUniformQuantizer(8, False)
        y, _ = obs.observe_quantize(t(w), q)
        for c in range(shape[0]):
            o1 = V.MinMaxObserver(False)
            s, z = o1.forward(t(w[c]))
            assert float(obs.scale[c]) == s and float(obs.zero_point[c]) == z
            G.assert_bitwise_f32(npy(y[c]), npy(V.UniformQuantizer(8, False).quantize(t(w[c]), s, z, False)),
                                 f"row {c}")


def _lsq_module(per_channel, config_act):
    if per_channel:
        return V.LSQFakeQuantize(learn_scale=True, config_act=config_act,
                                 observer=torch.quantization.MovingAveragePerChannelMinMaxObserver,
                                 quant_min=0, quant_max=255, dtype=torch.quint8,
                                 qscheme=torch.per_channel_affine, reduce_range=False,
                                 averaging_constant=0.01, ch_axis=1)
    return V.LSQFakeQuantize(learn_scale=True, config_act=config_act,
                             observer=torch.quantization.MovingAverageMinMaxObserver, quant_min=0,
                             quant_max=255, dtype=torch.quint8, qscheme=torch.per_tensor_affine,
                             reduce_range=False)


@pytest.mark.parametrize("case", G.cases("lsq_fake_quantize"), ids=lambda c: c["key"])
def test_golden_lsq_fake_quantize_on_cpu(case):
    """LSQFakeQuantize's learnable path on CPU tensors (host loops: per channel the [N, C, ...]
    rows of vsiq_host_pcm_*) == the reference goldens: y / grad_x bitwise, parameter
    gradients to the reference's fp32 sums (1e-4) and the oracle's f64 form (1e-9)."""
    fq = _lsq_module(case["per_channel"], case["config_act"])
    x, g = G.arr(case["x"]), G.arr(case["g"])
    fq(t(x))                                        # registers scale_param / zero_point_param_float
    fq.scale_param.data.copy_(t(G.arr(case["scale"])))
    fq.zero_point_param_float.data.copy_(t(G.arr(case["zp"])))
    fq.disable_observer()
    xg = t(x, grad=True)
    y = fq(xg)
    y.backward(t(g))
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")
    np.testing.assert_allclose(npy(fq.scale_param.grad), G.arr(case["scale_grad"]), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(npy(fq.zero_point_param_float.grad), G.arr(case["zp_grad"]), rtol=1e-4, atol=1e-6)
    if case["per_channel"]:
        s, z = G.arr(case["scale"]).reshape(-1), G.arr(case["zp"]).reshape(-1)
        gsc = O.lsq_module_grad_scale(x.shape, case["qmax"], True, case["config_act"])
        _, _, gso, gzo = O.pc_lsq_forward_backward(x, g, s, z, case["qmin"], case["qmax"], gsc, axis=1)
        np.testing.assert_allclose(npy(fq.scale_param.grad).reshape(-1), gso, rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(npy(fq.zero_point_param_float.grad).reshape(-1), gzo, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("shape,axis", [((6, 3, 7, 5), 1), ((2, 5, 7), 1), ((3, 5), 1), ((1, 4, 70000), 1),
                                        ((9, 16, 4, 4), 1), ((12, 27), 0), ((3, 70000), 0)])
def test_pc_lsq_host_vs_oracle(shape, axis):
    """host.PcLearnFn on either axis vs the oracle's pc_lsq_forward_backward: y / grad_x
    bitwise, f64 [C] gradients <= 1e-9 of the oracle's (f64 sums in another order)."""
    rng = np.random.default_rng(sum(shape) + axis)
    x = (rng.standard_normal(shape) * 2).astype(np.float32)
    g = rng.standard_normal(shape).astype(np.float32)
    C = shape[axis]
    s = rng.uniform(0.01, 0.1, C)
    z = np.rint(rng.uniform(0, 255, C)) + 0.2
    gscale = (255 * x.size / C) ** -0.5
    sp = torch.nn.Parameter(torch.tensor(s, dtype=torch.float64))
    zp = torch.nn.Parameter(torch.tensor(z, dtype=torch.float64))
    xg = t(x, grad=True)
    y = host.PcLearnFn.apply(xg, sp, zp, 0, 255, gscale, True, axis)
    y.backward(t(g))
    yo, gxo, gso, gzo = O.pc_lsq_forward_backward(x, g, s, z, 0, 255, gscale, axis=axis)
    G.assert_bitwise_f32(npy(y), yo, "y")
    G.assert_bitwise_f32(npy(xg.grad), gxo, "grad_x")
    np.testing.assert_allclose(npy(sp.grad), gso, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(npy(zp.grad), gzo, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("shape", [(4, 6, 5, 5), (2, 3, 70000)])
def test_lsq_fake_quantize_fixed_per_channel_on_cpu(shape):
    """LSQFakeQuantize with the observer's scale / zero_point buffers (no learning) on CPU:
    the host loops' per-channel fake quant == the reference's broadcast expression
    scale * (clamp(round(x / scale + zp)) - zp), bitwise; grad_x the STE mask."""
    rng = np.random.default_rng(11)
    x = (rng.standard_normal(shape) * 3).astype(np.float32)
    fq = V.LSQFakeQuantize(learn_scale=False, observer=torch.quantization.MovingAveragePerChannelMinMaxObserver,
                           quant_min=0, quant_max=255, dtype=torch.quint8, qscheme=torch.per_channel_affine,
                           ch_axis=1)
    fq(t(x))
    fq.disable_observer()
    xg = t(x, grad=True)
    y = fq(xg)
    view = [1, -1] + [1] * (len(shape) - 2)
    s, z = fq.scale.view(view), fq.zero_point.view(view)
    want = s * (torch.clamp(torch.round(t(x) / s + z), 0, 255) - z)
    G.assert_bitwise_f32(npy(y), npy(want), "y")
    gy = torch.ones_like(y)
    y.backward(gy)
    inr = (torch.round(t(x) / s + z) >= 0) & (torch.round(t(x) / s + z) <= 255)
    G.assert_bitwise_f32(npy(xg.grad), npy(inr.float()), "grad_x")


def test_host_pcm_abi_rejects_bad_channel_counts():
    lib = H.lib()
    x = torch.zeros(12)
    s = torch.ones(4, dtype=torch.float64)
    assert lib.vsiq_host_pcm_fq_fwd_f32(H.ptr(x), H.ptr(x), None, H.c_i64(6), H.c_i64(2), H.c_i64(4), H.ptr(s),
                                        None, 0, 0, 255) != 0   # 6 rows are not whole images of 4 channels
    assert lib.vsiq_host_pcm_fq_fwd_f32(H.ptr(x), H.ptr(x), None, H.c_i64(6), H.c_i64(2), H.c_i64(0), H.ptr(s),
                                        None, 0, 0, 255) != 0
    assert lib.vsiq_host_pcm_fq_fwd_f32(H.ptr(x), torch.empty(12).data_ptr(), None, H.c_i64(4), H.c_i64(3),
                                        H.c_i64(2), H.ptr(s), None, 0, 0, 255) == 0
