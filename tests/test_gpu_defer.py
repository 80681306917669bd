"""Deferred store phase (defer_stores, VSIQ_TUNE_STORE_DEFER) of the STE backward, and the
store gate (store_gate, VSIQ_TUNE_STORE_GATE) of K3 and the STE.

The deferral only changes when a workgroup's stores are issued, never what they hold:
the one-round 9-groups-per-lane path (automatic for 384..1024 workgroups) must equal
the plain kFlatU path bit for bit, and the oracle (oracle/fakequant_np.py
fq_backward_fixed / per_channel_backward_fixed / act_backward, reference
quantizers/uniform.py:54-55,95 autograd) on the same inputs.
"""
import numpy as np
import pytest
import torch

from vsiquantization_amd import _hip as H
from vsiquantization_amd import fakequant as FQ
from oracle import fakequant_np as O
from tests import goldens as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TUNE_STORE_DEFER = H.TUNE_STORE_DEFER


@pytest.fixture
def defer_tuning():
    H.set_tuning(H.TUNE_STORE_GATE, 0)   # the gate would take precedence on one-round grids
    yield lambda v: H.set_tuning(TUNE_STORE_DEFER, v)
    H.set_tuning(TUNE_STORE_DEFER, -1)
    H.set_tuning(H.TUNE_STORE_GATE, -1)


def _inputs(rows, rowlen, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((rows, rowlen)) * 0.05).astype(np.float32)
    g = rng.standard_normal((rows, rowlen)).astype(np.float32)
    g.flat[::9973] = np.nan
    g.flat[5::10007] = np.inf
    g.flat[7::8191] = np.float32(1e-41)   # denormal -> IEEE fallback group
    return x, g


@pytest.mark.parametrize("rows", [512, 768, 1024])
def test_per_channel_ste_deferred_equals_plain_and_oracle(rows, defer_tuning):
    rowlen = 9216
    x, g = _inputs(rows, rowlen, rows)
    scales = np.linspace(2e-4, 3e-3, rows)
    # per-row forward with clamping (tight scales) to get a non-trivial mask
    xd = torch.from_numpy(x).to(DEV)
    sd = torch.from_numpy(scales).to(DEV)
    _, mask, _ = FQ.per_channel_fake_quant(xd, sd, None, -128, 127, want_mask=True)
    m = G.unpack_mask(mask.cpu().numpy(), rows, rowlen)
    assert 0 < m.sum() < m.size
    gd = torch.from_numpy(g).to(DEV)
    outs = {}
    for v in (-1, 0, 3):
        defer_tuning(v)
        outs[v] = FQ.ste_backward(gd, mask, sd, rowlen).cpu().numpy()
    want = O.per_channel_backward_fixed(g, m, scales)
    for v, got in outs.items():
        G.assert_bitwise_f32(got, want, f"defer={v}")


@pytest.mark.parametrize("act", [None, "relu", "silu"])
def test_flat_ste_deferred_equals_plain(act, defer_tuning):
    n = 1024 * 9216   # one-round grid of 1024 workgroups: automatic deferral
    x, g = _inputs(1, n, 7)
    c = torch.from_numpy(x.reshape(-1) * 40).to(DEV)
    s = 0.021
    _, mask, _ = FQ.fake_quant(c, s, 0, -8, 7, want_mask=True, act=act)
    gd = torch.from_numpy(g.reshape(-1)).to(DEV)
    outs = {}
    for v in (-1, 0, 5):
        defer_tuning(v)
        outs[v] = FQ.ste_backward(gd, mask, s, pre=c if act else None, act=act).cpu().numpy()
    G.assert_bitwise_f32(outs[-1], outs[0], "auto vs plain")
    G.assert_bitwise_f32(outs[5], outs[0], "forced vs plain")
    if act is None:
        m = G.unpack_mask(mask.cpu().numpy(), 1, n).reshape(-1)
        G.assert_bitwise_f32(outs[-1], O.fq_backward_fixed(g.reshape(-1), m, s), "oracle")


@pytest.fixture
def gate_tuning():
    yield lambda v: H.set_tuning(H.TUNE_STORE_GATE, v)
    H.set_tuning(H.TUNE_STORE_GATE, -1)


@pytest.mark.parametrize("shape", [(1024, 9216), (2048, 4608), (700, 9216)])
def test_per_channel_store_gate_equals_plain_and_oracle(shape, gate_tuning):
    """K3 with the store gate (auto: one-round grids of >= 2 rows per CU; forced short
    and very long gates; off) and the STE with a forced gate: bit-identical outputs,
    qparams and masks, equal to the oracle (observers/minmax.py:32-74 per row, then
    quantizers/uniform.py:54-55,95)."""
    rows, rowlen = shape
    x, g = _inputs(rows, rowlen, rows + 1)
    xd = torch.from_numpy(x).to(DEV)
    gd = torch.from_numpy(g).to(DEV)
    outs = {}
    for v in (-1, 0, 300, 4000):
        gate_tuning(v)
        r = FQ.per_channel_observe_fq(xd, symmetric=False, qmin=0, qmax=255, want_codes=True, want_mask=True)
        gx = FQ.ste_backward(gd, r["mask"], r["scale"], rowlen)
        outs[v] = {k: r[k].cpu().numpy() for k in ("y", "codes", "mask", "scale", "zp")}
        outs[v]["gx"] = gx.cpu().numpy()
    ref = O.per_channel_observe_fq(x, False, 8, 8)
    m = G.unpack_mask(outs[0]["mask"], rows, rowlen)
    want_gx = O.per_channel_backward_fixed(g, ref["mask"], ref["scale"])
    for v, o in outs.items():
        G.assert_bitwise_f32(o["y"], ref["y"], f"y gate={v}")
        assert np.array_equal(o["scale"], ref["scale"]) and np.array_equal(o["zp"], ref["zp"].astype(np.float64))
        assert np.array_equal(o["codes"].astype(np.int64), ref["x_int"].astype(np.int64))
        assert np.array_equal(o["mask"], outs[0]["mask"])
        G.assert_bitwise_f32(o["gx"], want_gx, f"gx gate={v}")
    assert np.array_equal(m, ref["mask"].reshape(rows, rowlen))


@pytest.mark.parametrize("n,act", [(6_553_600, None), (6_553_600, "relu"), (13_107_200 + 4, "relu"),
                                   (4_800_000 + 3, None)])
def test_per_tensor_fq_store_gate_equals_plain_and_oracle(n, act, gate_tuning):
    """K1 / K5 forward on one-round 9-groups-per-lane grids with the store gate (auto, forced
    long) against the plain kFlatU grid (gate off): bit-identical y, codes and 1-bit masks,
    and y / codes / mask equal to the oracle (quantizers/uniform.py:54-55,95 after
    modules/fused.py:133's activation)."""
    rng = np.random.default_rng(n % 1000)
    c = (rng.standard_normal(n) * 0.3).astype(np.float32)
    c[::7919] = np.nan
    cd = torch.from_numpy(c).to(DEV)
    outs = {}
    for v in (0, -1, 4000):
        gate_tuning(v)
        y, mask, codes = FQ.fake_quant(cd, 0.021, 0, -8, 7, want_mask=True, want_codes=True, act=act)
        outs[v] = (y.cpu().numpy(), mask.cpu().numpy(), codes.cpu().numpy())
    for v in (-1, 4000):
        G.assert_bitwise_f32(outs[v][0], outs[0][0], f"y gate={v}")
        assert np.array_equal(outs[v][1], outs[0][1]) and np.array_equal(outs[v][2], outs[0][2])
    yo, qo, mo = O.fq_forward(O.act_forward(c, act), 0.021, 0, -8, 7)
    G.assert_bitwise_f32(outs[-1][0], yo, "y vs oracle")
    ok = ~np.isnan(qo)
    assert np.array_equal(outs[-1][2][ok].astype(np.int64), qo[ok].astype(np.int64))
    assert np.array_equal(G.unpack_mask(outs[-1][1], 1, n).reshape(-1), mo)


@pytest.mark.parametrize("shape", [(1024, 9216), (700, 4608), (1024, 8000)])
def test_per_channel_fixed_fq_store_gate_equals_plain_and_oracle(shape, gate_tuning):
    """Per-channel fake quant with given qparams (PerChannelUniformQuantizer / the
    learnable per-channel forward) on one-round 9-groups-per-lane grids behind the store
    gate vs the plain (rows, kFlatU chunks) grid: y, codes and masks bit for bit, and equal
    to the oracle (quantizers/uniform.py:54-55,95 per row)."""
    rows, rowlen = shape
    x, _ = _inputs(rows, rowlen, rows + 3)
    scales = np.linspace(2e-4, 3e-3, rows)
    zps = np.rint(np.linspace(100, 150, rows))
    xd = torch.from_numpy(x).to(DEV)
    sd = torch.from_numpy(scales).to(DEV)
    zd = torch.from_numpy(zps).to(DEV)
    outs = {}
    for v in (0, -1, 4000):
        gate_tuning(v)
        y, mask, codes = FQ.per_channel_fake_quant(xd, sd, zd, 0, 255, want_mask=True, want_codes=True)
        outs[v] = (y.cpu().numpy(), mask.cpu().numpy(), codes.cpu().numpy())
    for v in (-1, 4000):
        G.assert_bitwise_f32(outs[v][0], outs[0][0], f"y gate={v}")
        assert np.array_equal(outs[v][1], outs[0][1]) and np.array_equal(outs[v][2], outs[0][2])
    for r in (0, rows // 2, rows - 1):
        yo, qo, mo = O.fq_forward(x[r], float(scales[r]), float(zps[r]), 0, 255)
        G.assert_bitwise_f32(outs[-1][0][r], yo, f"y row {r}")
        assert np.array_equal(outs[-1][2][r].astype(np.int64), qo.astype(np.int64))
        assert np.array_equal(G.unpack_mask(outs[-1][1], rows, rowlen)[r], mo)
