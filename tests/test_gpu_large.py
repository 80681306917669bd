"""Maximum sizes: tensors of more than 2^31 elements (8.6 GB of fp32; the MI355X holds
288 GB) through K2 observe -> K1 fake quant (+ 1-bit mask) -> STE backward, the
learnable K1 + K4 pair, and the per-channel K3 forward, through the C ABI.

The oracle runs on slices the CPU finishes in seconds -- the head, a window across
element 2^31 (where a 32-bit element index would wrap) and the tail -- bit for bit;
the whole-tensor reductions are checked by size-independent properties: planted
extremes at the tail give the exact min/max and qparams (minmax.py:32-74), the mean|x|
statistic against torch's float64 sum, the LSQ scale gradient against the float64 sum
of the reference's fp32 autograd terms (uniform.py:47-56) restated in torch on the
device, chunk by chunk (IEEE fp32 division through float64, which rounds the same).
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
BIG = 2 ** 31 + 4100          # vector path (n % 4 == 0)
BIG_ODD = 2 ** 31 + 4099      # scalar tail path
W = 1 << 20


@pytest.fixture(autouse=True)
def _free():
    yield
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def windows(n):
    """[start, end) element windows; starts on 256-element mask-word boundaries."""
    mid = (1 << 31) - W // 2
    tail = ((n - W) // 256) * 256
    return [(0, W), (mid, min(n, mid + W)), (tail, n)]


def host(t, a, b):
    return t.reshape(-1)[a:b].cpu().numpy()


def mask_window(mask, a, b):
    """Bits of elements [a, b) of a flat (one-row) mask, a % 256 == 0."""
    words = mask.reshape(-1)[4 * (a // 256): 4 * (-(-b // 256))].cpu().numpy()
    return G.unpack_mask(words, 1, b - a)[0]


def randn(n, seed, std=1.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(n, generator=g, device=DEV).mul_(std)


@pytest.mark.parametrize("n", [BIG, BIG_ODD])
def test_observe_fq_ste_beyond_2g_elements(n):
    x = randn(n, 1)
    x[n - 1], x[n - 3] = 50.0, -40.0           # the extremes sit past element 2^31
    qp, st = FQ.observe_tensor(x, symmetric=False)
    s, z = O.minmax_qparams(-40.0, 50.0, False, 8)
    qph, sth = qp.cpu().numpy(), st.cpu().numpy()
    assert (qph[H.QP_MIN], qph[H.QP_MAX]) == (-40.0, 50.0)
    assert (qph[H.QP_SCALE], qph[H.QP_ZP]) == (s, z)
    assert sth[H.ST_N] == n
    want = float(torch.sum(x.abs(), dtype=torch.float64)) / n
    assert abs(sth[H.ST_MEANABS] - want) <= 1e-6 * want
    y, mask, _ = FQ.fake_quant(x, None, None, 0, 255, qp=qp, want_mask=True)
    g = x                                     # any gradient: reuse the input's memory
    gx = FQ.ste_backward(g, mask, s)
    torch.cuda.synchronize()
    for a, b in windows(n):
        xh = host(x, a, b)
        yo, _, mo = O.fq_forward(xh, s, z, 0, 255)
        G.assert_bitwise_f32(host(y, a, b), yo, f"y[{a}:{b}]")
        assert np.array_equal(mask_window(mask, a, b), mo), f"mask[{a}:{b}]"
        G.assert_bitwise_f32(host(gx, a, b), O.fq_backward_fixed(xh, mo, s), f"grad_x[{a}:{b}]")


def _lsq_grad_closed_form(x, g, s, qmin, qmax, gscale, chunk=1 << 28):
    """The reference's learnable autograd terms (uniform.py:47-56, zero point 0) in fp32,
    summed in float64 on the device: g*q and -(mask*g*s)*((x/s)/s)."""
    s64 = torch.tensor(s, dtype=torch.float64, device=DEV)
    s32 = s64.float()
    acc = torch.zeros((), dtype=torch.float64, device=DEV)
    for i in range(0, x.numel(), chunk):
        xc, gc = x[i:i + chunk], g[i:i + chunk]
        xs = (xc.double() / s32.double()).float()               # IEEE fp32 x / s
        r = torch.round(xs)
        q = r.clamp(qmin, qmax)
        gm = torch.where((r >= qmin) & (r <= qmax), gc * s32, torch.zeros_like(gc))
        xss = (xs.double() / s32.double()).float()
        acc += (gc * q).double().sum() + ((-gm) * xss).double().sum()
        del xs, r, q, gm, xss
    return float(acc) * gscale


def test_learnable_fq_lsq_beyond_2g_elements():
    n, s, qmin, qmax = BIG, 0.02, -128, 127
    x = randn(n, 2)
    g = randn(n, 3)
    gscale = O.grad_scale(qmax, n)
    y, _, _ = FQ.fake_quant(x, s, 0, qmin, qmax)
    gx, grads = FQ.lsq_backward(g, x, s, 0, qmin, qmax, gscale, False)
    torch.cuda.synchronize()
    for a, b in windows(n):
        yo, gxo, _, _ = O.lsq_forward_backward(host(x, a, b), host(g, a, b), s, 0, qmin, qmax, gscale)
        G.assert_bitwise_f32(host(y, a, b), yo, f"y[{a}:{b}]")
        G.assert_bitwise_f32(host(gx, a, b), gxo, f"grad_x[{a}:{b}]")
    del y, gx
    want = _lsq_grad_closed_form(x, g, s, qmin, qmax, gscale)
    got = float(grads[0])
    assert abs(got - want) <= 1e-9 * abs(want), (got, want)


def test_per_channel_observe_fq_beyond_2g_elements():
    """K3 over 256 rows of 8.4M elements (2^31 + 4096 in all): rows past element 2^31
    get their own min/max/qparams and fake quant, bit for bit."""
    C, L = 256, (1 << 23) + 16
    x = randn(C * L, 4, std=0.05).view(C, L)
    x[C - 1, L - 1] = 3.0                      # row 255 ends past 2^31
    out = FQ.per_channel_observe_fq(x, symmetric=False, qmin=0, qmax=255)
    y = out["y"]
    torch.cuda.synchronize()
    for c in (0, 127, 255):
        xr = x[c].cpu().numpy()
        o = O.per_channel_observe_fq(xr[None], False, 8)
        assert float(out["scale"][c]) == o["scale"][0] and float(out["zp"][c]) == o["zp"][0], c
        for a, b in ((0, W), (L - W, L)):
            G.assert_bitwise_f32(y[c, a:b].cpu().numpy(), o["y"][0, a:b], f"y[{c}, {a}:{b}]")
    assert float(out["run_max"][C - 1]) == 3.0


def test_deferred_records_beyond_2g_elements():
    """The deferred paths at the same size: K2p partial records + fold (calibration), the
    same tensor inside a K2m multi-tensor launch (records bit-identical), K2o (ReLU
    written + its records: exact min / max / n, y bitwise on the windows), and the
    records-only K4 backward + K4d fold against the one-launch K4 gradient."""
    from vsiquantization_amd.quantizers import deferred as D
    n = BIG
    x = randn(n, 5)
    x[n - 2], x[n - 5] = 60.0, -70.0
    parts = FQ.observe_parts(x)
    st = FQ.fold_parts(parts.view(1, -1))[0].cpu().numpy()
    assert (st[H.ST_MIN], st[H.ST_MAX], st[H.ST_N]) == (-70.0, 60.0, n)
    small = randn(1000, 6)
    outs = FQ.observe_parts_multi([small, x], None)
    assert torch.equal(outs[1], parts)
    del outs, parts
    # K2o (calibration's default kernel): ReLU(x) written and its records, past 2^31
    y, po = FQ.observe_parts_out(x, "relu")
    sto = FQ.fold_parts(po.view(1, -1))[0].cpu().numpy()
    assert (sto[H.ST_MIN], sto[H.ST_MAX], sto[H.ST_NAN], sto[H.ST_N]) == (0.0, 60.0, 0, n)
    torch.cuda.synchronize()
    for a, b in windows(n):
        G.assert_bitwise_f32(host(y, a, b), O.act_forward(host(x, a, b), "relu"), f"relu[{a}:{b}]")
    del y, po
    g = randn(n, 7)
    s, qmin, qmax = 0.05, -128, 127
    gscale = O.grad_scale(qmax, n)
    gx, grads = FQ.lsq_backward(g, x, s, 0, qmin, qmax, gscale, False)
    e = D._Fold()
    e.nrec = int(H.lib().vsiq_lsq_part_records(H.c_i64(n)))
    e.records = torch.empty(2 * e.nrec, dtype=torch.float64, device=DEV)
    gx2, e.zd, e.zh = D.lsq_backward_part(g, x, s, 0, qmin, qmax, False, None, e.records)
    e.gscale, e.qmin, e.qmax, e.learn_zp = gscale, qmin, qmax, False
    e.out = torch.empty(2, dtype=torch.float64, device=DEV)
    D.fold([e])
    assert torch.equal(gx, gx2)
    got, want = float(e.out[0]), float(grads[0])
    assert abs(got - want) <= 1e-12 * abs(want), (got, want)
