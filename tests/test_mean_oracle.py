"""mean|x| / mean x as the reference records them (quantization_manager.py:66-67,
torch.mean(torch.abs(x)).cpu().item() / torch.mean(x) on CPU tensors), and the learnable
scale built from them (qm.py:112, 2 * np.mean(mean_abs_x) / sqrt(2^(b-1) - 1)).

* oracle/mean_ref.c (torch's CPU cascade sum, then / float(n)) pinned bit for bit against
  torch.mean on this host: sizes around every boundary of the layout (vector, row,
  level step, GRAIN_SIZE, chunk), 1..16 threads; the vector width under
  ATEN_CPU_CAPABILITY=avx2 / default in a subprocess (the sum kernel is the AVX2 one on
  AVX-512 hosts too: V = 8 everywhere);
* the reference goldens: every recorded mean|x| / mean x of the manager sequences equals
  the oracle at the golden host's layout, and the golden init scale follows from them;
* the product's host loop (vsiq_host_torch_mean_f32, csrc/k_host.hip + mean_cascade.cuh)
  equals the oracle for every case, with the fused activations (ReLU, SiLU);
* QuantizationManager on CPU tensors under H.set_mean_reference: the calibrate ->
  init_scaling_factor_for_learning chain lands on the golden init scale bit for bit.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import fakequant_np as O
from tests import goldens as G

GOLDEN_THREADS = G.GOLDEN_SILU_REF[1]   # the golden host: 8 torch threads
SIZES = [0, 1, 3, 7, 8, 9, 31, 32, 33, 100, 511, 512, 513, 600, 8191, 8192, 8193, 32767, 32768, 32769,
         65536, 65537, 100_003, 262_144, 1 << 20, (1 << 20) + 13, 4_000_037]


@pytest.fixture
def threads():
    t0 = torch.get_num_threads()
    yield
    torch.set_num_threads(t0)


def _x(n, seed, scale=1.0):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal(n) * scale * rng.uniform(0.1, 10)).astype(np.float32)


def _same(a, b):
    a, b = np.float32(a), np.float32(b)
    return (np.isnan(a) and np.isnan(b)) or a.tobytes() == b.tobytes()


@pytest.mark.parametrize("nthreads", [1, 2, 3, 8, 16])
def test_oracle_equals_torch_mean(threads, nthreads):
    torch.set_num_threads(nthreads)
    bad = []
    for i, n in enumerate(SIZES):
        x = _x(n, 100 * nthreads + i)
        t = torch.from_numpy(x)
        for absf in (1, 0):
            want = (torch.mean(torch.abs(t)) if absf else torch.mean(t)).item()
            got = O.torch_mean(x, absf, nthreads)
            if not _same(got, want):
                bad.append((n, absf, float(got), want))
    assert not bad, bad[:5]


def test_oracle_specials(threads):
    torch.set_num_threads(4)
    x = _x(70_001, 7)
    x[[5, 900, 70_000]] = [np.inf, -0.0, 1e-40]
    for absf in (1, 0):
        t = torch.from_numpy(x)
        want = (torch.mean(torch.abs(t)) if absf else torch.mean(t)).item()
        assert _same(O.torch_mean(x, absf, 4), want)
    x[17] = np.nan
    assert np.isnan(O.torch_mean(x, 1, 4))


_CAP_SCRIPT = r"""
import sys, numpy as np, torch
sys.path.insert(0, {root!r})
from oracle import fakequant_np as O
bad = 0
for nt in (1, 5):
    torch.set_num_threads(nt)
    for i, n in enumerate([9, 100, 8193, 40_000, 300_001]):
        x = (np.random.default_rng(i).standard_normal(n) * 3).astype(np.float32)
        want = torch.mean(torch.abs(torch.from_numpy(x))).item()
        bad += np.float32(O.torch_mean(x, 1, nt)).tobytes() != np.float32(want).tobytes()
print(torch.backends.cpu.get_cpu_capability(), bad)
"""


@pytest.mark.parametrize("cap", ["avx2", "default"])
def test_oracle_vector_width_per_capability(cap):
    """The sum kernel's Vectorized<float> is 8 lanes whatever capability torch picks."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _CAP_SCRIPT.format(root=root)], capture_output=True, text=True,
                       env=dict(os.environ, ATEN_CPU_CAPABILITY=cap), timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split()[-1] == "0", r.stdout


def test_goldens_means_and_init_scale():
    """Every golden manager sequence: the recorded mean|x| / mean x are the oracle's at the
    golden host's layout, and init_scaling_factor_for_learning over the whole list (the
    calibration calls and the observe+quantize call) is the golden init scale, bitwise."""
    cases = G.cases("manager_sequence")
    assert cases
    for c in cases:
        xs = [G.arr(k) for k in c["xs"]]
        for i, x in enumerate(xs):
            assert _same(O.torch_mean(x, 1, GOLDEN_THREADS), c["calib"]["mean_abs_x"][i])
            assert _same(O.torch_mean(x, 0, GOLDEN_THREADS), c["calib"]["mean_x"][i])
        ms = [float(O.torch_mean(x, 1, GOLDEN_THREADS)) for x in xs + [G.arr(c["x_oq"])]]
        assert 2 * np.mean(ms) / np.sqrt(2 ** (c["bits"] - 1) - 1) == c["init_scale"]


@pytest.mark.parametrize("act", [None, "relu", "silu"])
@pytest.mark.parametrize("nthreads", [1, 3, 8])
def test_host_loop_equals_oracle(act, nthreads):
    """The product's host K11 (CPU tensors) against the oracle, bit for bit."""
    import vsiquantization_amd._hip as H
    from vsiquantization_amd.fakequant import torch_mean
    silu_ref = (32, nthreads)
    actv = H.SiluAct(*silu_ref) if act == "silu" else act
    for i, n in enumerate(SIZES):
        x = _x(n, 5000 + i)
        a = O.act_forward(x, act, silu_ref) if act else x
        got = torch_mean(torch.from_numpy(x), act=actv, ref=(8, nthreads)).numpy()
        for j, absf in enumerate((1, 0)):
            assert _same(got[j], O.torch_sum(a, absf, nthreads)), (n, absf, "sum")
            assert _same(got[2 + j], O.torch_mean(a, absf, nthreads)), (n, absf, "mean")


def test_manager_chain_host_golden_init_scale():
    """calibrate (observe only) -> observe+quantize -> init_scaling_factor_for_learning on
    CPU tensors under the golden host's mean reference: mean_abs_x, mean_x, std and the init
    scale are the reference's bits, with no value injected."""
    import vsiquantization_amd as V
    import vsiquantization_amd._hip as H
    H.set_mean_reference(GOLDEN_THREADS)
    try:
        for c in G.cases("manager_sequence"):
            qm = V.QuantizationManager("UniformQuantizer", "MinMaxObserver", c["bits"], c["sym"],
                                       is_learning_scale=True)
            qm.is_observer_qparam, qm.is_learning_scale, qm.is_quantize = True, False, False
            for k in c["xs"]:
                qm.quantize(torch.from_numpy(G.arr(k).copy()))
            assert [float(v) for v in qm.mean_abs_x] == c["calib"]["mean_abs_x"]
            assert [float(v) for v in qm.mean_x] == c["calib"]["mean_x"]
            assert [float(v) for v in qm.std] == c["calib"]["std"]   # the f64 std rounded to fp32
            qm.is_quantize = True
            qm.quantize(torch.from_numpy(G.arr(c["x_oq"]).copy()))
            qm.is_learning_scale = True
            qm.init_scaling_factor_for_learning()
            assert qm.scale == c["init_scale"]
    finally:
        H.clear_mean_reference()


def _std_restated(a):
    """torch CPU std of an fp32 tensor (ATen std_var_all_cpu): the fp32 torch.mean as a
    double, the f64 sum of squared deviations, / (n - 1), sqrt, rounded to fp32 once --
    what K11's std pass computes (csrc/k_mean.hip)."""
    a64 = a.astype(np.float64)
    m = float(torch.mean(torch.from_numpy(a)))
    return np.float32(np.sqrt(np.sum((a64 - m) ** 2) / (a.size - 1)))


@pytest.mark.parametrize("n", [2, 7, 600, 8193, 40_000, 1_000_003])
def test_std_restatement_equals_torch_std(n):
    """The restated std equals torch.std on this host bit for bit (the order of the f64 sum
    only moves it ~1e-16 relative, which the fp32 rounding absorbs)."""
    rng = np.random.default_rng(n)
    for scale, shift in ((1.0, 0.0), (0.05, 3.0), (10.0, -1.0)):
        a = (rng.standard_normal(n) * scale + shift).astype(np.float32)
        assert _std_restated(a).tobytes() == torch.std(torch.from_numpy(a)).numpy().tobytes(), (n, scale, shift)
