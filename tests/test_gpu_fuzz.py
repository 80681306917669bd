"""Seeded random-shape parity sweep through the C ABI (no fixed shapes): every launch
shape the dispatch can pick -- K3 register / long-row / gated one-round grids, the
STE's kFlatU / 9-group / gated forms, K1's kFlatU / gated 9-group forms, K4 at 4 and 8
groups per lane -- against the oracle (oracle/fakequant_np.py, which restates
observers/minmax.py:32-74 and quantizers/uniform.py:34-56,81-96 and their autograd).
Integer codes, y and grad_x bit-exact; learnable gradients <= 1e-9 of the f64 closed form.
"""
import numpy as np
import pytest
import torch

import vsiquantization_amd as V
from vsiquantization_amd import fakequant as FQ
from oracle import fakequant_np as O
from tests import goldens as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _shapes_pc(k, seed=11):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(k):
        rows = int(rng.choice([1, 3, 17, 255, 511, 700, 1024, 1100, 1600]))
        rowlen = int(rng.choice([1, 5, 27, 100, 576, 2304, 4608, 9216, 11000, 60000]))
        if rows * rowlen > 12_000_000:
            rowlen = max(1, 12_000_000 // rows)
        out.append((rows, rowlen, bool(rng.integers(2)), int(rng.choice([2, 4, 8]))))
    return out


@pytest.mark.parametrize("rows,rowlen,sym,bits", _shapes_pc(14))
def test_fuzz_per_channel_fwd_bwd(rows, rowlen, sym, bits):
    rng = np.random.default_rng(rows * 7919 + rowlen)
    w = (rng.standard_normal((rows, rowlen)) * rng.uniform(0.01, 3.0)).astype(np.float32)
    g = rng.standard_normal((rows, rowlen)).astype(np.float32)
    if rows > 2:
        w[rows // 2, :] = 0.0                      # zero row: scale 0 / eps edge
        w[rows // 3, rowlen // 2] = np.inf         # +inf element
    q = V.PerChannelUniformQuantizer(bits, sym)
    obs = V.PerChannelMinMaxObserver(sym)
    xg = torch.from_numpy(w).to(DEV).requires_grad_(True)
    y, _ = obs.observe_quantize(xg, q)
    y.backward(torch.from_numpy(g).to(DEV))
    ref = O.per_channel_observe_fq(w, sym, bits, 8)
    s, z = obs.get_scale_zero_point()
    assert np.array_equal(s.cpu().numpy(), ref["scale"])
    assert np.array_equal(z.cpu().numpy(), ref["zp"].astype(np.float64), equal_nan=True)
    G.assert_bitwise_f32(y.detach().cpu().numpy(), ref["y"], "y")
    G.assert_bitwise_f32(xg.grad.cpu().numpy(), O.per_channel_backward_fixed(g, ref["mask"], ref["scale"]), "gx")


def _sizes_flat(k, seed=12):
    rng = np.random.default_rng(seed)
    return [int(v) for v in rng.choice([5, 4097, 262_147, 2_000_000, 4_718_593, 6_553_600, 9_999_999,
                                        13_107_204, 21_000_000], size=k, replace=False)]


@pytest.mark.parametrize("n", _sizes_flat(7))
@pytest.mark.parametrize("act", [None, "relu"])
def test_fuzz_per_tensor_learnable(n, act):
    rng = np.random.default_rng(n % 100_003)
    x = (rng.standard_normal(n) * 0.7).astype(np.float32)
    g = rng.standard_normal(n).astype(np.float32)
    x[:: 104_729] = np.float32(3e-42)     # denormals -> IEEE division path for those groups
    scale, qmin, qmax = 0.037, -8, 7
    s = torch.nn.Parameter(torch.tensor(scale, dtype=torch.float64, device=DEV))
    xg = torch.from_numpy(x).to(DEV).requires_grad_(True)
    y = V.UniformQuantizer(4, True).quantize(xg, s, 0, True, act=act)
    y.backward(torch.from_numpy(g).to(DEV))
    xa = O.act_forward(x, act)
    yo, gxo, gso, _ = O.lsq_forward_backward(xa, g, scale, 0, qmin, qmax, O.grad_scale(qmax, n))
    G.assert_bitwise_f32(y.detach().cpu().numpy(), yo, "y")
    G.assert_bitwise_f32(xg.grad.cpu().numpy(), O.act_backward(gxo, x, act), "grad_x")
    assert float(s.grad) == pytest.approx(gso, rel=1e-9, abs=1e-12)
