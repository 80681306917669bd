"""K6 + LSQFakeQuantize / learnable per-channel on MI355X vs the reference goldens and
the oracle.  Bars: y and grad_x bit-exact; parameter gradients <= 1e-4 relative to
the reference's fp32 autograd sums, <= 1e-9 to the oracle's f64 closed form."""
import numpy as np
import pytest
import torch

import vsiquantization_amd as V
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


def _module(per_channel, config_act):
    if per_channel:
        return V.LSQFakeQuantize(learn_scale=True, config_act=config_act,
                                 observer=torch.quantization.MovingAveragePerChannelMinMaxObserver,
                                 quant_min=0, quant_max=255, dtype=torch.quint8,
                                 qscheme=torch.per_channel_affine, reduce_range=False,
                                 averaging_constant=0.01, ch_axis=1).to(DEV)
    return V.LSQFakeQuantize(learn_scale=True, config_act=config_act,
                             observer=torch.quantization.MovingAverageMinMaxObserver, quant_min=0,
                             quant_max=255, dtype=torch.quint8, qscheme=torch.per_tensor_affine,
                             reduce_range=False).to(DEV)


@pytest.mark.parametrize("case", G.cases("lsq_fake_quantize"), ids=lambda c: c["key"])
def test_golden_lsq_fake_quantize(case):
    fq = _module(case["per_channel"], case["config_act"])
    x = cu(G.arr(case["x"]))
    fq(x)                                           # registers scale_param / zero_point_param_float
    fq.scale_param.data.copy_(cu(G.arr(case["scale"])))
    fq.zero_point_param_float.data.copy_(cu(G.arr(case["zp"])))
    fq.disable_observer()
    xg = cu(G.arr(case["x"]), grad=True)
    y = fq(xg)
    y.backward(cu(G.arr(case["g"])))
    G.assert_bitwise_f32(npy(y), G.arr(case["y"]), "y")
    G.assert_bitwise_f32(npy(xg.grad), G.arr(case["grad_x"]), "grad_x")
    np.testing.assert_allclose(npy(fq.scale_param.grad), G.arr(case["scale_grad"]), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(npy(fq.zero_point_param_float.grad), G.arr(case["zp_grad"]), rtol=1e-4,
                               atol=1e-6)


@pytest.mark.parametrize("shape,axis", [((512, 3, 56, 56), 1), ((8, 64, 80, 80), 1), ((256, 27), 0),
                                        ((1024, 1024, 3, 3), 0), ((2, 5, 7), 1), ((3, 5), 1),
                                        # packed short rows (rowlen % 4 == 0, <= 2048): several
                                        # whole rows per workgroup, ragged last workgroup
                                        ((16, 32, 10, 10), 1), ((8, 16, 20, 20), 1), ((4, 8, 40, 40), 1),
                                        ((3, 7, 4), 1), ((2, 24, 32, 64), 1), ((1, 5, 12), 1),
                                        ((97, 3, 8), 1), ((300, 16), 0),
                                        # channel columns (K6 axis 1): several image blocks
                                        # per channel, a partial last one
                                        ((100, 8, 10, 10), 1), ((90, 4, 20, 20), 1), ((7, 3, 40, 48), 1),
                                        ((256, 16, 10, 10), 1)])
def test_pc_lsq_vs_oracle(shape, axis):
    rng = np.random.default_rng(sum(shape))
    x = (rng.standard_normal(shape) * 2).astype(np.float32)
    g = rng.standard_normal(shape).astype(np.float32)
    C = shape[axis]
    s = rng.uniform(0.01, 0.1, C)
    z = np.rint(rng.uniform(0, 255, C)) + 0.2
    gscale = (255 * x.size / C) ** -0.5
    sp = torch.nn.Parameter(torch.tensor(s, dtype=torch.float64, device=DEV))
    zp = torch.nn.Parameter(torch.tensor(z, dtype=torch.float64, device=DEV))
    xg = cu(x, grad=True)
    y = FQ.PerChannelLearnFn.apply(xg, sp, zp, 0, 255, gscale, True, axis)
    y.backward(cu(g))
    yo, gxo, gso, gzo = O.pc_lsq_forward_backward(x, g, s, z, 0, 255, gscale, axis=axis)
    G.assert_bitwise_f32(npy(y), yo, "y")
    G.assert_bitwise_f32(npy(xg.grad), gxo, "grad_x")
    np.testing.assert_allclose(npy(sp.grad), gso, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(npy(zp.grad), gzo, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("shape", [(16, 32, 10, 10), (3, 7, 4), (2, 24, 32, 64), (97, 3, 8), (100, 8, 10, 10),
                                   (256, 37, 10, 10), (9, 300, 6, 6)])
def test_packed_rows_equal_per_row_grid(shape):
    """Channel columns for K6 (VSIQ_TUNE_PC_PACKED 1, default; 10x10 rows in XCD-contiguous
    block order, VSIQ_TUNE_XCD_ORDER 0 the hardware order, 2 channel ranges per XCD) and
    packed short rows (2) vs
    one workgroup per row (0): y / grad_x bit for bit, per-channel gradients to float64
    reordering."""
    from vsiquantization_amd import _hip as H
    rng = np.random.default_rng(7)
    x = (rng.standard_normal(shape) * 2).astype(np.float32)
    g = rng.standard_normal(shape).astype(np.float32)
    C = shape[1]
    s = torch.tensor(rng.uniform(0.01, 0.1, C), dtype=torch.float64, device=DEV)
    z = torch.tensor(np.rint(rng.uniform(0, 255, C)) + 0.2, dtype=torch.float64, device=DEV)
    out = {}
    try:
        for packed, xo in ((1, 1), (1, 0), (1, 2), (2, 1), (0, 1)):
            H.set_tuning(H.TUNE_PC_PACKED, packed)
            H.set_tuning(H.TUNE_XCD_ORDER, xo)
            y = FQ.per_channel_fake_quant(cu(x), s, z, 0, 255, zp_round=True, axis=1)[0]
            gx, gs, gz = FQ.pc_lsq_backward(cu(g), cu(x), s, z, 0, 255, 1e-3, True, 1)
            out[packed if xo == 1 else -1 - xo] = [npy(t) for t in (y, gx, gs, gz)]
    finally:
        H.set_tuning(H.TUNE_PC_PACKED, 1)
        H.set_tuning(H.TUNE_XCD_ORDER, 2)   # the default
    for k in range(4):   # block order moves no record: every output identical, f64 included
        np.testing.assert_array_equal(out[-1][k], out[1][k])
        np.testing.assert_array_equal(out[-3][k], out[1][k])
    for mode in (1, 2):
        G.assert_bitwise_f32(out[mode][0], out[0][0], "y")
        G.assert_bitwise_f32(out[mode][1], out[0][1], "grad_x")
        np.testing.assert_allclose(out[mode][2], out[0][2], rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(out[mode][3], out[0][3], rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("shape,zpl", [((256, 16, 10, 10), True), ((100, 8, 10, 10), False), ((90, 4, 20, 20), True),
                                       ((7, 3, 40, 48), True), ((256, 37, 10, 10), False), ((3, 300, 8, 8), True)])
def test_pcc_in_launch_fold_equals_two_launch_fold(shape, zpl):
    """K6 on channel columns with the channel's last workgroup folding in the launch
    (vsiq_pcm_lsq_bwd_arrive_f32, what pc_lsq_backward calls) vs the separate fold
    launch (vsiq_pcm_lsq_bwd_f32): every output bit for bit, twice in a row (the
    counters are left zero), and the counters zero afterwards."""
    from vsiquantization_amd import _hip as H
    rng = np.random.default_rng(sum(shape))
    x = cu((rng.standard_normal(shape) * 2).astype(np.float32))
    g = cu(rng.standard_normal(shape).astype(np.float32))
    C = shape[1]
    s = torch.tensor(rng.uniform(0.01, 0.1, C), dtype=torch.float64, device=DEV)
    z = torch.tensor(np.rint(rng.uniform(0, 255, C)) + 0.2, dtype=torch.float64, device=DEV)
    rows, rowlen = x.numel() // (shape[2] * shape[3]), shape[2] * shape[3]
    a1 = [npy(t) for t in FQ.pc_lsq_backward(g, x, s, z, 0, 255, 1e-3, zpl, 1)]
    a2 = [npy(t) for t in FQ.pc_lsq_backward(g, x, s, z, 0, 255, 1e-3, zpl, 1)]
    gx = torch.empty_like(g)
    gs = torch.empty(C, dtype=torch.float64, device=DEV)
    gz = torch.empty(C, dtype=torch.float64, device=DEV)
    ws = torch.empty(int(H.lib().vsiq_pcm_workspace_doubles(rows, rowlen)), dtype=torch.float64, device=DEV)
    rc = H.lib().vsiq_pcm_lsq_bwd_f32(H.ptr(g), H.ptr(x), H.ptr(gx), H.c_i64(rows), H.c_i64(rowlen), H.c_i64(C),
                                      H.ptr(s), H.ptr(z), int(zpl), 0, 255, 1e-3, H.ptr(gs), H.ptr(gz), H.ptr(ws),
                                      H.c_i64(ws.numel()), H.stream_of(torch.device(DEV)))
    assert rc == 0
    b = [npy(t) for t in (gx, gs, gz)]
    for k in range(3):
        np.testing.assert_array_equal(a1[k], b[k])
        np.testing.assert_array_equal(a2[k], b[k])
    assert int(H.workspace(torch.device(DEV)).channel_counters(C).abs().sum()) == 0


def test_learnable_per_channel_quantizer_weights():
    """PerChannelUniformQuantizer learnable on an OIHW weight (axis 0, scale [C] f64)."""
    rng = np.random.default_rng(3)
    w = (rng.standard_normal((64, 32, 3, 3)) * 0.05).astype(np.float32)
    g = rng.standard_normal(w.shape).astype(np.float32)
    q = V.PerChannelUniformQuantizer(4, True)
    s = rng.uniform(0.005, 0.02, 64)
    sp = torch.nn.Parameter(torch.tensor(s, dtype=torch.float64, device=DEV))
    wg = cu(w, grad=True)
    y = q.quantize(wg, sp, 0, True)
    y.backward(cu(g))
    gscale = (q.qmax * w.size / 64) ** -0.5
    yo, gxo, gso, _ = O.pc_lsq_forward_backward(w, g, s, np.zeros(64), q.qmin, q.qmax, gscale, axis=0,
                                                learn_zp=False)
    G.assert_bitwise_f32(npy(y), yo, "y")
    G.assert_bitwise_f32(npy(wg.grad), gxo, "grad_w")
    np.testing.assert_allclose(npy(sp.grad), gso, rtol=1e-9, atol=1e-12)


def test_lsq_fake_quantize_axis_mismatch_raises_like_reference():
    fq = _module(True, False)
    fq(torch.randn(2, 6, 4, 4, device=DEV))
    fq.disable_observer()
    with pytest.raises(RuntimeError):
        fq(torch.randn(6, 5, 4, 4, device=DEV))    # weights with C_out != C_in


@pytest.mark.parametrize("shape,zpl", [((1024, 1024, 3, 3), True), ((256, 128, 3, 3), False),
                                       ((64, 32, 5, 5), True), ((300, 4000), False), ((40, 1030), True)])
def test_pc_lsq_axis0_row_resident_equals_two_stage_and_oracle(shape, zpl):
    """Axis-0 K6 with whole rows in registers (one launch, grad_scale/grad_zp per row
    written directly, store gate on one-round grids) vs the two-stage records + fold form
    (VSIQ_TUNE_PC_PACKED 0): grad_x bit for bit, per-channel gradients to float64
    reordering; both against the oracle (lsq_module.py:134-166 per channel)."""
    from vsiquantization_amd import _hip as H
    rng = np.random.default_rng(shape[0] + shape[1])
    x = (rng.standard_normal(shape) * 0.05).astype(np.float32)
    g = rng.standard_normal(shape).astype(np.float32)
    C = shape[0]
    s = rng.uniform(0.0005, 0.002, C)
    z = np.rint(rng.uniform(100, 150, C)) + 0.2 if zpl else np.zeros(C)
    gscale = (255 * x.size / C) ** -0.5
    sd = torch.tensor(s, dtype=torch.float64, device=DEV)
    zd = torch.tensor(z, dtype=torch.float64, device=DEV)
    out = {}
    try:
        for mode in (1, 0):
            H.set_tuning(H.TUNE_PC_PACKED, mode)
            gx, gs, gz = FQ.pc_lsq_backward(cu(g), cu(x), sd, zd, 0, 255, gscale, zpl, 0)
            out[mode] = [npy(t) for t in (gx, gs, gz)]
    finally:
        H.set_tuning(H.TUNE_PC_PACKED, 1)
    G.assert_bitwise_f32(out[1][0], out[0][0], "grad_x")
    np.testing.assert_allclose(out[1][1], out[0][1], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(out[1][2], out[0][2], rtol=1e-12, atol=1e-15)
    _, gxo, gso, gzo = O.pc_lsq_forward_backward(x, g, s, z, 0, 255, gscale, axis=0, learn_zp=zpl)
    G.assert_bitwise_f32(out[1][0], gxo, "grad_x vs oracle")
    np.testing.assert_allclose(out[1][1], gso, rtol=1e-9, atol=1e-12)
    if zpl:
        np.testing.assert_allclose(out[1][2], gzo, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("bits", [8, 4])
def test_manager_asym_per_channel_learnable_keeps_observer_zp(bits):
    """Asymmetric PerChannelUniformQuantizer through QuantizationManager: calibrate with
    PerChannelMinMaxObserver, activate learning -> the [C] scale becomes an f64 Parameter
    and the observer's per-channel zero points stay as fixed [C] tensors (not 0, which
    would clamp every negative weight at qmin = 0).  y / grad_w bitwise and the scale
    gradient <= 1e-9 vs the oracle with those zero points (learn_zp False)."""
    rng = np.random.default_rng(11 + bits)
    w = (rng.standard_normal((48, 16, 3, 3)) * 0.05).astype(np.float32)
    g = rng.standard_normal(w.shape).astype(np.float32)
    qm = V.QuantizationManager("PerChannelUniformQuantizer", "PerChannelMinMaxObserver", bits, False,
                               is_learning_scale=False).to(DEV)
    qm.is_quantize = False
    qm.quantize(cu(w))                                    # calibration: observe only
    s0 = npy(qm.scale).astype(np.float64)
    z0 = npy(qm.zero_point).astype(np.float64)
    assert z0.shape == (48,) and np.any(z0 > 0)
    qm.is_quantize = True
    qm.is_learning_scale = True
    qm.make_learn_qparameter()
    assert isinstance(qm.scale, torch.nn.Parameter) and qm.scale.dtype == torch.float64
    assert isinstance(qm.zero_point, torch.Tensor) and not qm.zero_point.requires_grad
    np.testing.assert_array_equal(npy(qm.zero_point), z0)
    wg = cu(w, grad=True)
    y = qm.quantize(wg)
    y.backward(cu(g))
    q = qm.quantizer
    gscale = (q.qmax * w.size / 48) ** -0.5
    yo, gxo, gso, _ = O.pc_lsq_forward_backward(w, g, s0, z0, q.qmin, q.qmax, gscale, axis=0,
                                                learn_zp=False)
    G.assert_bitwise_f32(npy(y), yo, "y")
    G.assert_bitwise_f32(npy(wg.grad), gxo, "grad_w")
    np.testing.assert_allclose(npy(qm.scale.grad), gso, rtol=1e-9, atol=1e-12)
    if bits == 8:
        assert npy(y).min() < 0, "negative weights must survive the asymmetric grid"
