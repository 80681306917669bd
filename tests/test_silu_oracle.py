"""Pin the oracle's SiLU restatement (oracle/silu_ref.c) against the reference's own
arithmetic: torch's CPU silu kernels, which is what F.silu in modules/fused.py:133 runs
on the reference's CPU tensors.  Bit-exact, at several sizes and torch thread counts --
which elements take glibc's scalar expf instead of the vectorized Sleef exp depends on
both (oracle/silu_ref.c header).  tests/golden/pin_silu.py runs the exhaustive 2^32
comparison of both exps (DESIGN.md §2.1 records its result).
"""
import numpy as np
import pytest
import torch

from oracle import fakequant_np as O

W = {"AVX512": 32, "AVX2": 16}.get(torch.backends.cpu.get_cpu_capability())
needs_vec = pytest.mark.skipif(W is None, reason="torch CPU kernels not AVX2/AVX-512 on this host")


@pytest.fixture
def threads():
    t0 = torch.get_num_threads()
    yield
    torch.set_num_threads(t0)


def _inputs(n, seed):
    rng = np.random.default_rng(seed)
    c = (rng.standard_normal(n) * 4).astype(np.float32)
    if n > 40:   # specials and the ranges where both exps saturate / underflow
        c[:12] = [0.0, -0.0, np.nan, np.inf, -np.inf, 1e-40, -1e-40, 88.5, -88.5, 104.5, -104.5, 17.3]
    return c, rng.standard_normal(n).astype(np.float32)


def _bits_equal(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a.view(np.uint32)[~na], b.view(np.uint32)[~nb])


@needs_vec
@pytest.mark.parametrize("n", [1, 31, 33, 1000, 1296, 32767, 32768, 32769, 100_003, 1_000_000])
@pytest.mark.parametrize("nt", [1, 3, 8])
def test_silu_oracle_equals_torch_cpu(n, nt, threads):
    torch.set_num_threads(nt)
    c, g = _inputs(n, n + nt)
    want_y = torch.nn.functional.silu(torch.from_numpy(c)).numpy()
    want_g = torch.ops.aten.silu_backward(torch.from_numpy(g), torch.from_numpy(c)).numpy()
    ref = (W, torch.get_num_threads())
    assert _bits_equal(O.silu_forward(c, ref), want_y)
    assert _bits_equal(O.silu_backward(g, c, ref), want_g)


@needs_vec
def test_silu_reference_depends_on_thread_count(threads):
    """The irreducible part: the reference's own F.silu bits change with torch's thread
    count (chunk remainders move), so parity is defined per (vector width, threads)."""
    c, _ = _inputs(1_000_003, 5)
    outs = []
    for nt in (1, 3, 7):
        torch.set_num_threads(nt)
        outs.append(torch.nn.functional.silu(torch.from_numpy(c)).numpy())
    assert not (_bits_equal(outs[0], outs[1]) and _bits_equal(outs[0], outs[2]))
    for nt, y in zip((1, 3, 7), outs):
        assert _bits_equal(O.silu_forward(c, (W, nt)), y)


def test_scalar_map_layout():
    """at::parallel_for chunking: serial below 32768 elements; remainder of every chunk."""
    m = O.silu_scalar_map(1000, (32, 8))
    assert m.sum() == 1000 % 32 and m[-(1000 % 32):].all()
    m = O.silu_scalar_map(100_003, (32, 3))   # chunks of 33335, 33335, 33333: 23 + 23 + 21
    assert m.sum() == 23 + 23 + 21 and m[33335 - 23:33335].all() and not m[33335 - 24]
    assert O.silu_scalar_map(100_003, (32, 1)).sum() == 100_003 % 32
    assert not O.silu_scalar_map(4096, (32, 8)).any()
    assert not O.silu_scalar_map(1001, (0, 8)).any()


def test_exps_differ_where_it_matters():
    """Sleef and glibc expf disagree on a few % of activation-range inputs: the scalar
    path cannot be approximated by the vector one."""
    x = np.linspace(-12, 12, 200_001, dtype=np.float32)
    a, b = O.exp_sleef_glibc(x)
    frac = float(np.mean(a != b))
    assert 0.001 < frac < 0.1
    # both within one ulp of the correctly rounded value
    cr = np.exp(x.astype(np.float64)).astype(np.float32)
    for e in (a, b):
        d = np.abs(e.view(np.int32).astype(np.int64) - cr.view(np.int32).astype(np.int64))
        assert d.max() <= 1
