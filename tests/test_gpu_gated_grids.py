"""The one-round gated grids of round 5 against the oracle / the un-gated kernels, at the
sizes that select them and with the variants the benches do not run: K1 (flat 2-groups
grid gated at 1.6M..4.2M elements, 9-groups grid at 4.7M..18.9M) with the 1-bit mask and
the uint8 codes, misaligned views; K2o (the same two forms) on misaligned views with
every activation; records-only K4d (2 groups per lane gated up to 4.2M, 4 per lane from
~50M) with the SiLU backward and a learned zero point.  The gate is a delay only: every
output is compared bit for bit (records: min / max / NaN / n exactly, sums to f64 order).
Reference: quantizers/uniform.py:34-56, 81-96; observers/minmax.py:42-47."""
import numpy as np
import pytest
import torch

from vsiquantization_amd import _hip as H
from vsiquantization_amd import fakequant as FQ
from vsiquantization_amd.quantizers import deferred as D
from oracle import fakequant_np as O
from tests import goldens as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

# 1.6M (flat gated), 3.3M + 5 (flat gated, ragged), 6.6M (9-groups gated), 13.1M + 3
SIZES = [1_638_400, 3_276_805, 6_553_600, 13_107_203]


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    H.lib()
    H.set_silu_reference(32, 8)
    yield
    H.set_silu_reference()


def _x(n, seed, misaligned):
    rng = np.random.default_rng(seed)
    a = (rng.standard_normal(n + 1) * 2.5).astype(np.float32)
    a[5:9] = [np.nan, -0.0, 0.0, 1e-40]
    t = torch.from_numpy(a).to(DEV)
    return (t[1:], a[1:]) if misaligned else (t[:n].clone(), a[:n])


@pytest.mark.parametrize("misaligned", [False, True])
@pytest.mark.parametrize("n", SIZES)
def test_k1_gated_grids_mask_codes_vs_oracle(n, misaligned):
    x, a = _x(n, n % 101, misaligned)
    s, z, qmin, qmax = 0.031, 3.0, -8, 7
    for _ in range(3):   # the first launches of a site time candidate gates
        y, mask, codes = FQ.fake_quant(x, s, z, qmin, qmax, want_mask=True, want_codes=True)
    yo, qo, mo = O.fq_forward(a, s, z, qmin, qmax)
    G.assert_bitwise_f32(y.cpu().numpy(), yo, "y")
    assert np.array_equal(G.unpack_mask(mask.cpu().numpy(), 1, n)[0], mo)
    ok = ~np.isnan(qo)
    assert np.array_equal(codes.cpu().numpy()[ok].astype(np.int64), qo[ok].astype(np.int64))


@pytest.mark.parametrize("act", [None, "relu", "silu"])
@pytest.mark.parametrize("n", SIZES)
def test_k2o_gated_grids_misaligned(n, act):
    x, _ = _x(n, n % 89, True)
    want = FQ.fold_parts(FQ.observe_parts(x, act=act).reshape(1, -1))
    for _ in range(3):
        y, parts = FQ.observe_parts_out(x, act)
    got = FQ.fold_parts(parts.reshape(1, -1))
    exact = [H.ST_MIN, H.ST_MAX, H.ST_NAN, H.ST_N]
    assert torch.equal(got[0, exact], want[0, exact])
    torch.testing.assert_close(got, want, rtol=1e-12, atol=0.0, equal_nan=True)
    ref = FQ.activation(x, act) if act else x
    G.assert_bitwise_f32(y.cpu().numpy(), ref.cpu().numpy(), "y")


@pytest.mark.parametrize("act", ["silu", "relu"])
@pytest.mark.parametrize("learn_zp", [False, True])
@pytest.mark.parametrize("n", [1_638_403, 3_276_800, 52_428_800])
def test_k4d_gated_grids_equal_k4(n, act, learn_zp):
    """Records-only K4d (gated 2-groups grids up to 4.2M, 4 groups per lane from ~50M)
    folded == the in-kernel-fold K4 (grad_x bitwise, grads to f64 order)."""
    rng = np.random.default_rng(n % 997 + int(learn_zp))
    x = torch.from_numpy((rng.standard_normal(n) * 0.4).astype(np.float32)).to(DEV)
    g = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(DEV)
    qmin, qmax = (0, 15) if learn_zp else (-8, 7)
    sd = torch.tensor(0.05, dtype=torch.float64, device=DEV)
    zd = torch.tensor(7.3, dtype=torch.float64, device=DEV) if learn_zp else 0.0
    gscale = (qmax * n) ** -0.5
    gx_ref, grads_ref = FQ.lsq_backward(g, x, sd, zd, qmin, qmax, gscale, learn_zp, act=act)
    for _ in range(3):
        e = D._Fold()
        e.nrec = int(H.lib().vsiq_lsq_part_records(H.c_i64(n)))
        e.records = torch.full((2 * e.nrec,), float("nan"), dtype=torch.float64, device=DEV)
        gx, e.zd, e.zh = D.lsq_backward_part(g, x, sd, zd, qmin, qmax, learn_zp, act, e.records)
        e.gscale, e.qmin, e.qmax, e.learn_zp = gscale, qmin, qmax, learn_zp
        e.out = torch.empty(2, dtype=torch.float64, device=DEV)
        e.keep = (sd, zd)
        D.fold([e])
    torch.cuda.synchronize()
    assert torch.equal(gx.view(torch.int32), gx_ref.view(torch.int32))
    np.testing.assert_allclose(e.out.cpu().numpy(), grads_ref.cpu().numpy(), rtol=1e-12, atol=1e-300)
