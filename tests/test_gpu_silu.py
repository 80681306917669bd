"""SiLU bit for bit as the reference computes it (F.silu on CPU tensors, modules/fused.py:133):
every kernel that applies a fused SiLU (K5: K1 / STE / K4 / K4d / K2 / K2p / K2m / K8 / K9,
and the activation alone) against

* this box's own torch CPU kernels (torch.nn.functional.silu / aten.silu_backward) at
  several thread counts -- the product follows the host's torch layout by default;
* the oracle (oracle/silu_ref.c) under pinned multi-chunk layouts (W = 32 / 16 elements
  per vectorized step, 7 threads), where every chunk of the tensor has a scalar
  remainder computed with glibc's expf;
* the two exps themselves (vsiq_selftest_exp_f32) on 2^24 inputs across the whole
  activation range, the overflow / underflow edges and random bit patterns.
"""
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
HOST_W = {"AVX512": 32, "AVX2": 16}.get(torch.backends.cpu.get_cpu_capability())


def cu(a, grad=False):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    return t.requires_grad_(True) if grad else t


def npy(t):
    return t.detach().cpu().numpy()


@pytest.fixture
def pin():
    """Pin the product's SiLU layout (and restore host-following + torch threads after)."""
    t0 = torch.get_num_threads()

    def _pin(w, t):
        H.set_silu_reference(w, t)
        return (w, t)
    yield _pin
    H.set_silu_reference()
    torch.set_num_threads(t0)


def _inputs(n, seed, scale=4.0):
    rng = np.random.default_rng(seed)
    c = (rng.standard_normal(n) * scale).astype(np.float32)
    if n > 16:
        c[:10] = [0.0, -0.0, np.nan, np.inf, -np.inf, 1e-40, 88.9, -88.9, 104.5, -104.5]
    return c, rng.standard_normal(n).astype(np.float32)


def test_exps_bitwise_vs_oracle():
    x = np.concatenate([
        np.linspace(-110.0, 110.0, 1 << 23, dtype=np.float32),
        np.linspace(-1.0, 1.0, 1 << 22, dtype=np.float32),
        np.random.default_rng(0).integers(0, 2**32, 1 << 22, dtype=np.uint64).astype(np.uint32).view(np.float32),
        np.array([np.inf, -np.inf, np.nan, 0.0, -0.0, 88.72283, 88.72284, -103.97208, -103.97209, 100.0, 100.00001,
                  -104.0, -104.00001, 1e-45, -1e-45], np.float32)])
    xs = cu(x)
    ys, yg = torch.empty_like(xs), torch.empty_like(xs)
    H.check(H.lib().vsiq_selftest_exp_f32(H.ptr(xs), H.ptr(ys), H.ptr(yg), H.c_i64(x.size), H.stream_of(torch.device(DEV))),
            "vsiq_selftest_exp_f32")
    ws, wg = O.exp_sleef_glibc(x)
    G.assert_bitwise_f32(npy(ys), ws, "Sleef expf_u10")
    G.assert_bitwise_f32(npy(yg), wg, "glibc expf")


@pytest.mark.skipif(HOST_W is None, reason="this host's torch CPU kernels are neither AVX2 nor AVX-512")
@pytest.mark.parametrize("threads", [1, 5, 16])
@pytest.mark.parametrize("n", [1, 31, 1296, 32769, 100_003, 1_000_003, 4_000_037])
def test_activation_equals_host_torch_cpu(n, threads, pin):
    """Default layout = this host's torch: the HIP activation equals torch's CPU F.silu and
    silu_backward on the same values, bit for bit, at every thread count."""
    torch.set_num_threads(threads)
    c, g = _inputs(n, n + threads)
    x = cu(c, grad=True)
    y = FQ.activation(x, "silu")
    y.backward(cu(g))
    want_y = torch.nn.functional.silu(torch.from_numpy(c)).numpy()
    want_g = torch.ops.aten.silu_backward(torch.from_numpy(g), torch.from_numpy(c)).numpy()
    G.assert_bitwise_f32(npy(y), want_y, "silu")
    G.assert_bitwise_f32(npy(x.grad), want_g, "silu_backward")


LAYOUTS = [(32, 7), (16, 7), (32, 1), (0, 1)]
SIZES = [33, 40_000, 100_003, 1_000_003]


@pytest.mark.parametrize("ref", LAYOUTS, ids=lambda r: f"W{r[0]}T{r[1]}")
@pytest.mark.parametrize("n", SIZES)
def test_fixed_fq_and_ste_vs_oracle(n, ref, pin):
    pin(*ref)
    c, g = _inputs(n, n)
    y, mask, _ = FQ.fake_quant(cu(c), 0.021, 3, 0, 255, want_mask=True, act="silu")
    gc = FQ.ste_backward(cu(g), mask, 0.021, pre=cu(c), act="silu")
    a = O.act_forward(c, "silu", ref)
    yo, _, mo = O.fq_forward(a, 0.021, 3, 0, 255)
    G.assert_bitwise_f32(npy(y), yo, "y")
    assert np.array_equal(G.unpack_mask(npy(mask), 1, n)[0], mo)
    G.assert_bitwise_f32(npy(gc), O.act_backward(O.fq_backward_fixed(g, mo, 0.021), c, "silu", ref), "grad_c")


@pytest.mark.parametrize("ref", LAYOUTS[:2], ids=lambda r: f"W{r[0]}T{r[1]}")
@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("deferred", [False, True])
def test_learnable_vs_oracle(n, ref, deferred, pin):
    """K1 + K4 (and the records-only K4d with its fold) through a fused SiLU."""
    pin(*ref)
    c, g = _inputs(n, n + 1, 2.0)
    c[2:5] = [0.5, 7.0, -7.0]   # finite: a NaN / inf term would make the scale gradient NaN
    q = V.UniformQuantizer(8, True)
    s = torch.nn.Parameter(torch.tensor(0.03, dtype=torch.float64, device=DEV))
    x = cu(c, grad=True)
    if deferred:
        from vsiquantization_amd.quantizers.deferred import DeferredLearnFn, QParamBundleFn
        sb = QParamBundleFn.apply(s)
        sb = sb[0] if isinstance(sb, tuple) else sb
        y = DeferredLearnFn.apply(x, sb, 0, q.qmin, q.qmax, O.grad_scale(q.qmax, n), False, "silu")
    else:
        y = q.quantize(x, s, 0, True, act="silu")
    y.backward(cu(g))
    a = O.act_forward(c, "silu", ref)
    yo, gxo, gso, _ = O.lsq_forward_backward(a, g, 0.03, 0, q.qmin, q.qmax, O.grad_scale(q.qmax, n))
    G.assert_bitwise_f32(npy(y), yo, "y")
    G.assert_bitwise_f32(npy(x.grad), O.act_backward(gxo, c, "silu", ref), "grad_c")
    assert abs(float(s.grad) - gso) <= 1e-9 * abs(gso)


@pytest.mark.parametrize("ref", LAYOUTS[:2], ids=lambda r: f"W{r[0]}T{r[1]}")
@pytest.mark.parametrize("n", SIZES)
def test_observers_vs_oracle(n, ref, pin):
    """K2 (per-call), K2p records + fold, K2m, and K8 / K9 (observe + fake quant)."""
    pin(*ref)
    c, _ = _inputs(n, n + 2, 3.0)
    c[2:5] = [0.5, 7.0, -7.0]   # no NaN in silu(c) (silu(-inf) is NaN): the qparams exist
    a = O.act_forward(c, "silu", ref)
    mn, mx = O.observe_minmax(a)
    s, z = O.minmax_qparams(mn, mx, False, 8)
    x = cu(c)
    qp, st = FQ.observe_tensor(x, symmetric=False, act="silu")
    qph = npy(qp)
    assert (qph[H.QP_SCALE], qph[H.QP_ZP], qph[H.QP_MIN], qph[H.QP_MAX]) == (s, z, mn, mx)
    folded = npy(FQ.fold_parts(torch.stack([FQ.observe_parts(x, act="silu")])))[0]
    assert (folded[H.ST_MIN], folded[H.ST_MAX]) == (mn, mx)
    multi = FQ.observe_parts_multi([x, x[: n // 2]], None, act="silu")
    single = FQ.observe_parts(x, act="silu")
    assert torch.equal(multi[0].view(torch.int64), single.view(torch.int64))
    if n <= FQ.observe_fq_parts_max_elems():
        y, qp2, _, _, _ = FQ.observe_fake_quant(x, symmetric=False, qmin=0, qmax=255, act="silu")
        assert (float(qp2[H.QP_SCALE]), float(qp2[H.QP_ZP])) == (s, z)
        G.assert_bitwise_f32(npy(y), O.fq_forward(a, s, z, 0, 255)[0], "K8/K9 y")
    # the half-size tensor has its own chunk layout
    h = n // 2
    mh, xh = O.observe_minmax(O.act_forward(c[:h], "silu", ref))
    fh = npy(FQ.fold_parts(torch.stack([multi[1]])))[0]
    assert (fh[H.ST_MIN], fh[H.ST_MAX]) == (mh, xh)


def test_calibration_forward_hands_on_reference_silu(pin):
    """A calibration forward (observe only) returns silu(c) for the next layer: the HIP
    activation, torch CPU's bits (not torch's HIP silu)."""
    ref = pin(32, 3)
    qm = V.QuantizationManager("UniformQuantizer", "MinMaxObserver", 8, True)
    qm.is_quantize, qm.is_learning_scale, qm.is_observer_qparam = False, False, True
    c, _ = _inputs(200_003, 9)
    c[2:5] = [0.25, 7.0, -7.0]
    out = qm.quantize(cu(c), act="silu")
    G.assert_bitwise_f32(npy(out), O.act_forward(c, "silu", ref), "calibration output")
    qm._join()
    mn, mx = O.observe_minmax(O.act_forward(c, "silu", ref))
    assert (qm.observer.min_val, qm.observer.max_val) == (mn, mx)


def test_silu_act_code_layout():
    """The act argument carries (W, threads); malformed codes are rejected by the ABI."""
    H.set_silu_reference(32, 12)
    try:
        code = H.act_code("silu")
        assert code == 2 | (32 << 8) | (12 << 16)
        x = torch.randn(100, device=DEV)
        y = torch.empty_like(x)
        assert H.lib().vsiq_act_fwd_f32(H.ptr(x), H.ptr(y), H.c_i64(100), 2 | (24 << 8), H.stream_of(torch.device(DEV))) != 0
        assert H.lib().vsiq_act_fwd_f32(H.ptr(x), H.ptr(y), H.c_i64(100), 1 | (32 << 8), H.stream_of(torch.device(DEV))) != 0
        assert H.lib().vsiq_act_fwd_f32(H.ptr(x), H.ptr(y), H.c_i64(100), code, H.stream_of(torch.device(DEV))) == 0
    finally:
        H.set_silu_reference()


@pytest.mark.parametrize("act", ["relu", "silu", None])
@pytest.mark.parametrize("n", [7, 4096, 100_003, 3 * 2**20 + 4, 4_718_592, 6_553_600, 13_107_203, 18_874_368,
                               26 * 2**20 + 3])
def test_observe_parts_out_equals_act_then_parts(n, act, pin):
    """K2o (vsiq_act_observe_part_out_f32): y = act(c) and the deferred records in one
    pass.  y == the activation alone == the oracle, bit for bit; the folded records ==
    K2p's fold in min / max / NaN count / n exactly and in the sums to float64 summation
    order (one record per one-shot workgroup instead of one per grid-stride wave); the
    legacy grid-stride form (VSIQ_TUNE_K2O_FORM 1) gives K2p's records bit for bit.
    4.7M..18.9M elements take the one-round gated form (C5's 6.6M / 13M layers; its
    bounds: 2 and 8 workgroups per CU of 9 groups per lane)."""
    pin(32, 7)
    c, _ = _inputs(n, n + 5)
    x = cu(c)
    y, parts = FQ.observe_parts_out(x, act)
    assert parts.numel() == FQ.part_out_slot_doubles(n)
    want_parts = FQ.observe_parts(x, act=act)
    got, want = FQ.fold_parts(parts.reshape(1, -1)), FQ.fold_parts(want_parts.reshape(1, -1))
    exact = [H.ST_MIN, H.ST_MAX, H.ST_NAN, H.ST_N]
    assert torch.equal(got[0, exact], want[0, exact])
    torch.testing.assert_close(got, want, rtol=1e-12, atol=0.0, equal_nan=True)
    G.assert_bitwise_f32(npy(y), npy(FQ.activation(x, act) if act else x), "y")
    if n < 2**22:
        G.assert_bitwise_f32(npy(y), O.act_forward(c, act, (32, 7)) if act else c, "y vs oracle")
    lib = H.lib()
    assert lib.vsiq_set_tuning(H.TUNE_K2O_FORM, 1) == 0
    try:
        y1, parts1 = FQ.observe_parts_out(x, act)
        assert torch.equal(parts1.view(torch.int64), want_parts.view(torch.int64))
        assert torch.equal(y1.view(torch.int32), y.view(torch.int32))
    finally:
        assert lib.vsiq_set_tuning(H.TUNE_K2O_FORM, 0) == 0


@pytest.mark.parametrize("block", [256, 512, 1024])
@pytest.mark.parametrize("groups", [1, 2, 4, 8, 16])
def test_observe_parts_out_every_group_count(groups, block):
    """Every one-shot K2o groups-per-lane instance (VSIQ_TUNE_K2O_GROUPS) on a ragged,
    misaligned-tail tensor: y bitwise, folded min / max / NaN exact and sums to f64
    order against K2p."""
    lib = H.lib()
    c, _ = _inputs(5 * 2**20 + 13, groups)
    c = np.nan_to_num(c, nan=0.5, posinf=50.0, neginf=-50.0)   # finite: the sums are compared too
    x = cu(c)
    want = FQ.fold_parts(FQ.observe_parts(x, act="relu").reshape(1, -1))
    assert lib.vsiq_set_tuning(H.TUNE_K2O_GROUPS, groups) == 0
    assert lib.vsiq_set_tuning(H.TUNE_K2O_BLOCK, block) == 0
    try:
        y, parts = FQ.observe_parts_out(x, "relu")
        assert parts.numel() == lib.vsiq_observe_part_out_records(H.c_i64(x.numel())) * H.PART_LEN
        assert parts.numel() == -(-x.numel() // (4 * block * groups)) * H.PART_LEN
    finally:
        assert lib.vsiq_set_tuning(H.TUNE_K2O_GROUPS, 0) == 0
        assert lib.vsiq_set_tuning(H.TUNE_K2O_BLOCK, 0) == 0
    got = FQ.fold_parts(parts.reshape(1, -1))
    exact = [H.ST_MIN, H.ST_MAX, H.ST_NAN, H.ST_N]
    assert torch.equal(got[0, exact], want[0, exact])
    torch.testing.assert_close(got, want, rtol=1e-12, atol=0.0, equal_nan=True)
    G.assert_bitwise_f32(npy(y), npy(FQ.activation(x, "relu")), "y")   # CPU relu: -0.0 kept


def test_silu_layout_recorded_with_qparams_survives_checkpoint(pin):
    """A manager records the SiLU reference layout (W, torch threads) at its first SiLU
    call and keeps using it: a state_dict saved from a run at 16 torch threads and loaded
    into a process at 1 thread reproduces the 16-thread bits (forward and the SiLU
    backward), with a warning; without the record the 1-thread layout gives other bits."""
    H.set_silu_reference()   # follow this host's torch
    n = 16 * 40000 + 12      # 16 chunks at 16 threads, one serial run at 1: different scalar tails
    c, g = _inputs(n, 77)
    x, gy = cu(c), cu(g)

    def manager():
        qm = V.QuantizationManager("UniformQuantizer", "MinMaxObserver", 8, True, is_learning_scale=False)
        return qm

    def learn(qm):
        qm.is_learning_scale, qm.is_quantize = True, True
        if not isinstance(qm.scale, torch.Tensor):   # a fresh manager (the checkpoint brings the value)
            qm.scale = torch.tensor(0.1, dtype=torch.float64, device=DEV)
        qm.make_learn_qparameter()

    def run(qm):
        xi = x.clone().requires_grad_(True)
        y = qm.quantize(xi, act="silu")
        y.backward(gy)
        torch.cuda.synchronize()
        return npy(y), npy(xi.grad)

    torch.set_num_threads(16)
    a = manager()
    a.is_observer_qparam, a.is_quantize = True, False
    a.quantize(x, act="silu")
    a.init_scaling_factor_for_learning()
    learn(a)
    assert a.silu_layout == (HOST_W or 16, 16)
    y16, gx16 = run(a)
    sd = a.state_dict()
    assert tuple(sd["silu_layout"].tolist()) == a.silu_layout
    torch.set_num_threads(1)
    b = manager()
    learn(b)
    b.load_state_dict(sd)
    assert b.silu_layout == a.silu_layout
    with pytest.warns(RuntimeWarning, match="SiLU reference layout"):
        yb, gxb = run(b)
    G.assert_bitwise_f32(yb, y16, "y")
    G.assert_bitwise_f32(gxb, gx16, "grad_x")
    ctrl = manager()
    learn(ctrl)
    ctrl.load_state_dict({k: v for k, v in sd.items() if k != "silu_layout"})
    _, gxc = run(ctrl)
    assert ctrl.silu_layout == (HOST_W or 16, 1)
    assert not np.array_equal(gxc.view(np.uint32), gx16.view(np.uint32))
