"""The CPU baseline (oracle/eager_torch.py, the reference's eager op sequence) is pinned
to the reference goldens too, so bench.py's cpu_baseline times the same arithmetic the
GPU path is checked against."""
import pytest
import torch

from oracle import eager_torch as E
from oracle.fakequant_np import minmax_qparams, qrange
from tests.goldens import arr, assert_bitwise_f32, cases


@pytest.mark.parametrize("c", cases("fixed_fq"), ids=lambda c: c["key"])
def test_eager_fixed(c):
    qmin, qmax = qrange(c["bits"], c["sym"])
    x = torch.from_numpy(arr(c["x"])).requires_grad_(True)
    y = E.fake_quant(x, c["scale"], c["zp"], qmin, qmax)
    y.backward(torch.from_numpy(arr(c["g"])))
    assert_bitwise_f32(y.detach().numpy(), arr(c["y"]), "y")
    assert_bitwise_f32(x.grad.numpy(), arr(c["grad_x"]), "grad_x")


@pytest.mark.parametrize("c", cases("per_tensor_observe_fq"), ids=lambda c: c["key"])
def test_eager_observe(c):
    x = torch.from_numpy(arr(c["x"]))
    mn, mx = E.observe(x)
    assert (mn, mx) == (c["min_val"], c["max_val"])
    if "raises" in c or c.get("scale") is None:
        return  # the reference raises in round(); covered by test_oracle_golden
    s, z = minmax_qparams(mn, mx, c["sym"], c["obs_bits"])
    assert (s, z) == (c["scale"], c["zp"])
    qmin, qmax = qrange(c["bits"], c["sym"])
    assert_bitwise_f32(E.fake_quant(x, s, z, qmin, qmax).numpy(), arr(c["y"]), "y")


@pytest.mark.parametrize("c", [c for c in cases("per_channel_observe_fq") if not c["special"]],
                         ids=lambda c: c["key"])
def test_eager_per_channel(c):
    w = torch.from_numpy(arr(c["x"]))
    gx = E.per_channel_step(w, torch.from_numpy(arr(c["g"])), c["sym"], c["bits"])
    assert_bitwise_f32(gx.numpy(), arr(c["grad_x"]), "grad_x")


@pytest.mark.parametrize("c", [c for c in cases("learnable_fq") if c["sym"]], ids=lambda c: c["key"])
def test_eager_lsq(c):
    x = torch.from_numpy(arr(c["x"]))
    gx, gs = E.lsq_step(x, torch.from_numpy(arr(c["g"])), scale=c["scale"], bits=c["bits"])
    assert_bitwise_f32(gx.numpy(), arr(c["grad_x"]), "grad_x")
    assert abs(float(gs) - c["scale_grad"]) <= 1e-6 * max(1.0, abs(c["scale_grad"]))


def test_lsq_step_asym_matches_oracle():
    """The asymmetric learnable step (LSQQuantizer: learnable zero point through
    zero_point_rounding, uniform.py:47-56, 98-102) -- bench.py's C3 --asym CPU baseline --
    against the oracle's closed form: grad_x bitwise, scale / zp gradients to 1e-4."""
    import numpy as np
    import torch
    from oracle import eager_torch as E
    from oracle import fakequant_np as O
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(4, 3, 16, 16, generator=gen)
    g = torch.randn(4, 3, 16, 16, generator=gen)
    gx, gs, gz = E.lsq_step(x, g, scale=0.03, bits=8, zero_point=3.0)
    _, gxo, gso, gzo = O.lsq_forward_backward(x.numpy(), g.numpy(), 0.03, 3.0, 0, 255,
                                              (255 * x.numel()) ** -0.5, learn_zp=True)
    assert np.array_equal(gx.numpy().view(np.uint32), gxo.view(np.uint32))
    np.testing.assert_allclose(float(gs), gso, rtol=1e-4)
    np.testing.assert_allclose(float(gz), gzo, rtol=1e-4)
