"""Calibration on MI355X: side-stream (async) observers give exactly the synchronous
results; the fused-ReLU observer path through calibrate_qat_model."""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

from vsiquantization_amd.modules.fused import ConvBn, ConvBnReLU
from vsiquantization_amd.utils.quantize_manager import calibrate_qat_model, data_calib

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _model():
    torch.manual_seed(0)
    layers = []
    for cin, cout in ((3, 16), (16, 32), (32, 32)):
        cv = nn.Conv2d(cin, cout, 3, padding=1, bias=False)
        bn = nn.BatchNorm2d(cout)
        bn.running_var.uniform_(0.5, 2.0)
        layers.append(ConvBnReLU(cv, bn, nn.ReLU(), "MinMaxObserver", "UniformQuantizer", "MinMaxObserver",
                                 "UniformQuantizer", True, True, True, 4, 4))
    return nn.Sequential(*layers).to(DEV)


def _loader(n=6):
    g = torch.Generator().manual_seed(1)
    return [(torch.randint(0, 256, (4, 3, 32, 32), generator=g, dtype=torch.uint8), None) for _ in range(n)]


def _state(model):
    out = []
    for m in model:
        for qm in (m.weight_quantizer, m.activation_quantizer):
            out.append((qm.observer.min_val, qm.observer.max_val, list(qm.mean_abs_x), list(qm.mean_x),
                        list(qm.std)))
    return out


def test_async_observers_equal_sync():
    a = _model()
    b = copy.deepcopy(a)
    calibrate_qat_model(a, _loader(), data_calib, DEV, async_observers=True, defer_observers=False)
    calibrate_qat_model(b, _loader(), data_calib, DEV, async_observers=False, defer_observers=False)
    sa, sb = _state(a), _state(b)
    assert sa == sb
    assert all(len(s[2]) == 6 for s in sa)
    # the flag is restored and nothing stays pending
    assert all(not m.activation_quantizer.async_observer for m in a)
    assert all(m.activation_quantizer._side is None for m in a)


def test_deferred_calibration_equals_sync():
    """defer_observers (K2p partial records + one fold + replay at the end) gives the
    reference's running min/max and qparams exactly, and its mean|x| / mean / std lists."""
    a = _model()
    b = copy.deepcopy(a)
    calibrate_qat_model(a, _loader(), data_calib, DEV)   # default: deferred
    calibrate_qat_model(b, _loader(), data_calib, DEV, defer_observers=False)
    sa, sb = _state(a), _state(b)
    for x, y in zip(sa, sb):
        assert (x[0], x[1]) == (y[0], y[1])
        for i in (2, 3, 4):
            np.testing.assert_allclose(x[i], y[i], rtol=1e-6, atol=0)
    for ma, mb in zip(a, b):
        for qa, qb in ((ma.weight_quantizer, mb.weight_quantizer),
                       (ma.activation_quantizer, mb.activation_quantizer)):
            assert float(qa.scale) == float(qb.scale)
            assert float(qa.zero_point) == float(qb.zero_point)
            assert not qa.dist_defer and not qa._pending_records


@pytest.mark.parametrize("act", [None, "relu", "silu"])
@pytest.mark.parametrize("n", [1, 7, 4096, 1000003, 3 * 2**20 + 5, 13107200])
def test_observe_parts_fold_equals_k2(n, act):
    """K2p slots folded in one launch == the K2 per-call stats record: min/max/nan/n
    exact, sums to float64 reordering."""
    from vsiquantization_amd import _hip as H
    from vsiquantization_amd import fakequant as FQ
    g = torch.Generator(device=DEV).manual_seed(n)
    xs = [torch.randn(n, device=DEV, generator=g) * 3 for _ in range(3)]
    xs[1][n // 2] = float("nan")
    xs.append(torch.randn(n + 1, device=DEV, generator=g)[1:])   # misaligned view
    stride = FQ.part_slot_doubles()
    slots = torch.full((len(xs), stride), float("nan"), dtype=torch.float64, device=DEV)
    for i, x in enumerate(xs):
        FQ.observe_parts(x, out=slots[i], act=act)
    got = FQ.fold_parts(slots).cpu()
    for i, x in enumerate(xs):
        _, st = FQ.observe_tensor(x, symmetric=True, want_qp=False, act=act)
        want = st.cpu()
        exact = [H.ST_MIN, H.ST_MAX, H.ST_NAN, H.ST_N]
        assert torch.equal(got[i, exact], want[exact]), (i, got[i], want)
        np.testing.assert_allclose(got[i, H.ST_SUMABS:H.ST_SUMSQ + 1].numpy(),
                                   want[H.ST_SUMABS:H.ST_SUMSQ + 1].numpy(), rtol=1e-12, atol=1e-300)
        np.testing.assert_allclose(got[i, H.ST_MEANABS:].numpy(), want[H.ST_MEANABS:].numpy(),
                                   rtol=1e-6, equal_nan=True)


def test_fold_parts_unwritten_slot_folds_nothing():
    from vsiquantization_amd import _hip as H
    from vsiquantization_amd import fakequant as FQ
    stride = FQ.part_slot_doubles()
    slots = torch.zeros(2, stride, dtype=torch.float64, device=DEV)
    slots[1, 7] = 1e30   # garbage record count: ignored, never read out of range
    st = FQ.fold_parts(slots).cpu()
    assert torch.all(st[:, H.ST_N] == 0)
    assert torch.all(torch.isinf(st[:, H.ST_MIN])) and torch.all(st[:, H.ST_MIN] > 0)


@pytest.mark.parametrize("act", [None, "relu", "silu"])
def test_observe_parts_multi_records_bitwise_equal_per_call(act):
    """K2m (vsiq_act_observe_part_multi_f32): every tensor's partial records are the
    same bits as its own K2p launch -- 40 tensors (two launches of 32 + 8) of mixed
    sizes across all three groups-per-lane classes, ragged n, a misaligned view, NaNs."""
    from vsiquantization_amd import fakequant as FQ
    g = torch.Generator(device=DEV).manual_seed(3)
    sizes = [1, 7, 4096, 1000003, 3 * 2**20 + 5, 13107200, 52428800, 65536, 999, 2**20]
    xs = [torch.randn(sizes[i % len(sizes)] + (i // len(sizes)), device=DEV, generator=g) * (1 + i)
          for i in range(39)]
    xs[5][3] = float("nan")
    xs.append(torch.randn(4097, device=DEV, generator=g)[1:])   # misaligned view
    per = [FQ.observe_parts(x, act=act) for x in xs]
    multi = FQ.observe_parts_multi(xs, None, act=act)
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(per, multi)):
        assert a.numel() == b.numel()
        assert torch.equal(a.view(torch.int64), b.view(torch.int64)), i


@pytest.mark.parametrize("act", [None, "relu"])
def test_observe_parts_multi_all_vector_batch_bitwise(act):
    """A batch whose tensors all take the 16-byte path launches K2m's all-vector variant
    (84 VGPRs, no scalar-path code): records still the same bits as per-call K2p, over
    every groups-per-lane class and the whole / partial last step of each tensor."""
    from vsiquantization_amd import fakequant as FQ
    g = torch.Generator(device=DEV).manual_seed(5)
    sizes = [4, 4096, 1000004, 3 * 2**20 + 4, 13107200, 52428800, 65536, 2**20, 6553600, 409600]
    xs = [torch.randn(n, device=DEV, generator=g) * 3 for n in sizes]
    xs[2][17] = float("nan")
    per = [FQ.observe_parts(x, act=act) for x in xs]
    multi = FQ.observe_parts_multi(xs, None, act=act)
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(per, multi)):
        assert torch.equal(a.view(torch.int64), b.view(torch.int64)), i


def test_queued_deferred_calibration_equals_unqueued(monkeypatch):
    """QuantizationManager's deferred calls queued and observed by K2m (opt-in,
    VSIQ_OBSERVE_BATCH=1) give the same running min/max, qparams and stats lists, bit for
    bit, as the default (fused layers: K2o, act + records in one pass; others: K2p)."""
    a = _model()
    b = copy.deepcopy(a)
    monkeypatch.setenv("VSIQ_OBSERVE_BATCH", "1")
    calibrate_qat_model(a, _loader(), data_calib, DEV)
    monkeypatch.delenv("VSIQ_OBSERVE_BATCH")
    calibrate_qat_model(b, _loader(), data_calib, DEV)
    assert _state(a) == _state(b)
    from vsiquantization_amd import observe_batch
    assert observe_batch.pending() == 0


def test_queued_observer_detects_in_place_change():
    from vsiquantization_amd import observe_batch
    from vsiquantization_amd.fakequant import part_slot_doubles
    x = torch.randn(1000, device=DEV)
    slot = torch.empty(part_slot_doubles(x.numel()), dtype=torch.float64, device=DEV)
    observe_batch.add(x, None, slot)
    x.mul_(2)
    with pytest.raises(RuntimeError, match="modified in place"):
        observe_batch.flush()
    assert observe_batch.pending() == 0


@pytest.mark.parametrize("act", [None, "relu", "silu"])
@pytest.mark.parametrize("sym,qmin,qmax", [(True, -128, 127), (False, 0, 255), (True, -8, 7), (False, 0, 3)])
@pytest.mark.parametrize("n", [1, 7, 255, 256, 4097, 65535, 65536, 65537, 262143, 262144])
@pytest.mark.parametrize("parts", [None, False, True, "k10"])
def test_observe_fq_small_equals_observe_then_fq(n, sym, qmin, qmax, act, parts):
    """K8 (vsiq_act_observe_fq_f32: observe + qparams + fake quant of a small tensor in one
    launch) == K2 (vsiq_act_observe_f32) then K1 (vsiq_act_fq_fwd_f32 on its qparams
    record): running state, qparams record, y, codes and the 1-bit mask bit for bit, the
    stats sums to float64 reordering; three calls carry the running state (one with a NaN,
    which changes nothing, minmax.py:42-47); misaligned input takes the scalar path.
    The same for K9 (vsiq_act_observe_fq_parts_f32: K2p records, then every fake-quant
    workgroup folds them; parts=True, and the default above 16384 elements) and K10
    (vsiq_act_observe_fq_grid_f32, the one-launch form with a grid barrier; parts="k10")."""
    from vsiquantization_amd import _hip as H
    from vsiquantization_amd import fakequant as FQ
    if parts is False and n > FQ.observe_fq_max_elems():
        pytest.skip("K8 takes at most observe_fq_max_elems()")
    g = torch.Generator(device=DEV).manual_seed(n + qmax)
    xs = [torch.randn(n, device=DEV, generator=g) * (1 + i) for i in range(3)]
    if n > 1:
        xs[1][n // 2] = float("nan")
    xs.append(torch.randn(n + 1, device=DEV, generator=g)[1:])     # misaligned view
    ra = torch.zeros(2, device=DEV)
    rb = torch.zeros(2, device=DEV)
    for x in xs:
        y, qp, st, mask, codes = FQ.observe_fake_quant(x, symmetric=sym, qmin=qmin, qmax=qmax, run_minmax=ra,
                                                       act=act, want_mask=True, want_codes=True, parts=parts)
        qp2, st2 = FQ.observe_tensor(x, symmetric=sym, run_minmax=rb, act=act)
        y2, mask2, codes2 = FQ.fake_quant(x, None, None, qmin, qmax, qp=qp2, want_mask=True, want_codes=True,
                                          act=act)
        torch.cuda.synchronize()
        assert torch.equal(ra.view(torch.int32), rb.view(torch.int32))
        assert torch.equal(qp.view(torch.int64), qp2.view(torch.int64))
        assert torch.equal(y.view(torch.int32), y2.view(torch.int32))
        assert torch.equal(mask, mask2) and torch.equal(codes, codes2)
        exact = [H.ST_MIN, H.ST_MAX, H.ST_NAN, H.ST_N]
        assert torch.equal(st[exact], st2[exact])
        np.testing.assert_allclose(st.cpu().numpy(), st2.cpu().numpy(), rtol=1e-12, atol=1e-300, equal_nan=True)


@pytest.mark.parametrize("act", [None, "relu", "silu"])
@pytest.mark.parametrize("n", [16385, 20000, 65536, 65537, 100003, 131072, 200000, 262144])
def test_k10_grid_barrier_equals_k9(n, act):
    """K10 (one launch, grid barrier) == K9 (two launches) bit for bit -- y, codes, mask,
    running state, qparams AND the stats record (the same K2p records folded in the same
    order) -- over calls of different grid sizes back to back on one stream (the barrier
    words are reset by the last workgroup out), and the barrier's counter words are zero
    afterwards with no timed-out waits (counter word 35)."""
    from vsiquantization_amd import _hip as H
    from vsiquantization_amd import fakequant as FQ
    g = torch.Generator(device=DEV).manual_seed(n)
    ra = torch.zeros(2, device=DEV)
    rb = torch.zeros(2, device=DEV)
    for m in (n, 16385 + n % 977, n):   # alternate grid sizes on the same counter words
        for i in range(2):
            x = torch.randn(m, device=DEV, generator=g) * (1 + i)
            if i:
                x[m // 3] = float("nan")
            a = FQ.observe_fake_quant(x, symmetric=False, qmin=0, qmax=255, run_minmax=ra, act=act,
                                      want_mask=True, want_codes=True, parts="k10")
            b = FQ.observe_fake_quant(x, symmetric=False, qmin=0, qmax=255, run_minmax=rb, act=act,
                                      want_mask=True, want_codes=True, parts="k9")
            torch.cuda.synchronize()
            assert torch.equal(ra.view(torch.int32), rb.view(torch.int32))
            for u, v in zip(a, b):
                assert torch.equal(u.view(torch.uint8), v.view(torch.uint8))
    w = H.workspace(DEV, n)
    assert w.counter[33:36].cpu().tolist() == [0, 0, 0]


def test_k10_graph_replay_equals_eager():
    """K10 captured in a HIP graph and replayed (BASELINE C1's launch mode in bench.py):
    the same bits as eager, the barrier words zero after the replays."""
    from vsiquantization_amd import _hip as H
    from vsiquantization_amd import fakequant as FQ
    x = torch.randn(256, 256, device=DEV)
    ra = torch.zeros(2, device=DEV)
    y0, qp0, st0, _, _ = FQ.observe_fake_quant(x, symmetric=True, qmin=-128, qmax=127, run_minmax=ra, parts="k10")
    s = torch.cuda.Stream(DEV)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        rb = torch.zeros(2, device=DEV)
        FQ.observe_fake_quant(x, symmetric=True, qmin=-128, qmax=127, run_minmax=rb, parts="k10")   # workspace of s
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            out = FQ.observe_fake_quant(x, symmetric=True, qmin=-128, qmax=127, run_minmax=rb, parts="k10")
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        rb.zero_()
        graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out[0].view(torch.int32), y0.view(torch.int32))
    assert torch.equal(out[1].view(torch.int64), qp0.view(torch.int64))
    assert torch.equal(out[2].view(torch.int64), st0.view(torch.int64))
    assert torch.equal(rb, ra)
    for w in list(H._WS.values()):   # every stream's and capture's barrier words
        assert int(w.counter[33:36].abs().sum()) == 0


def test_observe_fq_small_rejects_large():
    from vsiquantization_amd import fakequant as FQ
    n = FQ.observe_fq_max_elems() + 1
    with pytest.raises(Exception):
        FQ.observe_fake_quant(torch.randn(n, device=DEV), symmetric=True, qmin=-128, qmax=127, parts=False)
    n = FQ.observe_fq_parts_max_elems() + 1
    with pytest.raises(Exception):
        FQ.observe_fake_quant(torch.randn(n, device=DEV), symmetric=True, qmin=-128, qmax=127)


@pytest.mark.parametrize("sym,bits", [(True, 8), (False, 8), (True, 4)])
@pytest.mark.parametrize("shape", [(256, 256), (7, 13, 41, 43)])
def test_manager_observe_quantize_mid_size_vs_oracle(shape, sym, bits):
    """QuantizationManager per-call observe + quantize (qm.py:73-90 -> minmax.py:32-74 ->
    uniform.py:34-56) at BASELINE C1's 256x256 and an odd 157K-element shape, both on the
    K9 path: three calls carry the running min/max (the second with a NaN, which changes
    nothing), then y, the running bounds, scale / zero point and the STE gradient of the
    last call bit for bit against the oracle."""
    import vsiquantization_amd as V
    from oracle import fakequant_np as O
    rng = np.random.default_rng(sum(shape) + bits)
    qm = V.QuantizationManager("UniformQuantizer", "MinMaxObserver", bits, sym, True)
    qm.is_observer_qparam, qm.is_learning_scale, qm.is_quantize = True, False, True
    mn, mx = 0, 0
    for i in range(3):
        x = (rng.standard_normal(shape) * (1 + i)).astype(np.float32)
        if i == 1:
            x.reshape(-1)[x.size // 3] = np.nan
        g = rng.standard_normal(shape).astype(np.float32)
        xt = torch.from_numpy(x).to(DEV).requires_grad_(True)
        y = qm.quantize(xt)
        y.backward(torch.from_numpy(g).to(DEV))
        mn, mx = O.observe_minmax(x, mn, mx)
        s, z = O.minmax_qparams(mn, mx, sym, 8)   # the manager's observer is always 8-bit
        qmin, qmax = O.qrange(bits, sym)
        yo, _, mask = O.fq_forward(x, s, z, qmin, qmax)
        gxo = O.fq_backward_fixed(g, mask, s)
        torch.cuda.synchronize()
        assert (qm.observer.min_val, qm.observer.max_val) == (mn, mx)
        assert float(qm.scale) == s and float(qm.zero_point) == z
        assert np.array_equal(y.detach().cpu().numpy().view(np.uint32), yo.view(np.uint32))
        assert np.array_equal(xt.grad.cpu().numpy().view(np.uint32), gxo.view(np.uint32))


class _Residual(nn.Module):
    """Observed layers whose outputs user code modifies in place afterwards: a residual
    ``+=`` on a ConvBn output (no activation: the observed tensor is the one handed back),
    an in-place ReLU and an in-place scale on fused-ReLU outputs."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(2)
        names = ("MinMaxObserver", "UniformQuantizer", "MinMaxObserver", "UniformQuantizer")

        def bn(c):
            b = nn.BatchNorm2d(c)
            b.running_var.uniform_(0.5, 2.0)
            return b
        self.a = ConvBnReLU(nn.Conv2d(3, 16, 3, padding=1, bias=False), bn(16), nn.ReLU(), *names, True, True,
                            True, 4, 4)
        self.b = ConvBn(nn.Conv2d(16, 16, 3, padding=1, bias=False), bn(16), *names, True, True, True, 4, 4)
        self.c = ConvBnReLU(nn.Conv2d(16, 16, 3, padding=1, bias=False), bn(16), nn.SiLU(), *names, True, True,
                            True, 4, 4)
        self.act = nn.ReLU(inplace=True)

    def forward(self, x):
        y = self.a(x)
        z = self.b(y)
        z += y              # residual, in place on an observed (handed back) tensor
        z = self.act(z)     # in-place ReLU
        w = self.c(z)
        w.mul_(0.5)         # in place on a fused layer's calibration output
        return w

    def layers(self):
        return [self.a, self.b, self.c]


def test_deferred_calibration_with_in_place_ops_equals_sync():
    """deferred calibration (the default) must observe each call before user
    code can modify the tensor in place -- the result equals the per-call observers'."""
    a = _Residual().to(DEV)
    b = copy.deepcopy(a)
    calibrate_qat_model(a, _loader(), data_calib, DEV)
    calibrate_qat_model(b, _loader(), data_calib, DEV, defer_observers=False)
    sa, sb = _state(a.layers()), _state(b.layers())
    for x, y in zip(sa, sb):
        assert (x[0], x[1]) == (y[0], y[1])
        for i in (2, 3, 4):
            np.testing.assert_allclose(x[i], y[i], rtol=1e-6, atol=1e-7)
    from vsiquantization_amd import observe_batch
    assert observe_batch.pending() == 0
