"""Reads during the default (deferred) calibration see the reference's per-call state.

The reference updates ``qm.scale / zero_point / mean_abs_x / mean_x / std`` and the
observer's ``min_val / max_val`` on every call (quantizers/quantization_manager.py:55-71,
observers/minmax.py:42-47), and ``data_calib`` is user code that may read them between
batches (utils/quantize_manager.py:4-31).  The deferred calibration (K2p / K2o records,
one sync at the end) folds a manager's pending calls on the first read instead; these
tests check each read against the oracle replayed call by call and against the per-call
path, and that the end state does not depend on whether anything was read.
"""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

import vsiquantization_amd as V
from vsiquantization_amd import _hip as H
from vsiquantization_amd.distributed import sync_calibration
from vsiquantization_amd.modules.fused import ConvBnReLU
from vsiquantization_amd.utils.quantize_manager import calibrate_qat_model, data_calib
from oracle import fakequant_np as O
from tests import goldens as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    H.lib()


def _deferred_manager(bits, sym):
    qm = V.QuantizationManager("UniformQuantizer", "MinMaxObserver", bits, sym, True)
    qm.is_observer_qparam, qm.is_learning_scale, qm.is_quantize = True, False, False
    qm.dist_defer = True
    return qm


def _read(qm):
    obs = qm.observer
    return dict(scale=float(qm.scale), zero_point=float(qm.zero_point), min_val=obs.min_val,
                max_val=obs.max_val, qp=obs.get_scale_zero_point(), mean_abs_x=list(qm.mean_abs_x),
                mean_x=list(qm.mean_x), std=list(qm.std))


def _assert_read_equal(got, want):
    for k in ("scale", "zero_point", "min_val", "max_val", "qp"):
        assert got[k] == want[k], (k, got[k], want[k])
    for k in ("mean_abs_x", "mean_x", "std"):
        assert len(got[k]) == len(want[k]), k
        np.testing.assert_allclose(got[k], want[k], rtol=1e-6, atol=1e-7, err_msg=k)


@pytest.mark.parametrize("act", [None, "relu"])
@pytest.mark.parametrize("case", G.cases("manager_sequence"), ids=lambda c: c["key"])
def test_deferred_reads_after_each_call_equal_oracle(case, act):
    """One manager in deferred mode (weight path K2p for act None, fused-activation K2o
    for "relu"); every attribute read after each call equals the oracle replayed up to
    that call; the end state equals the reference golden (act None) and a manager that
    was never read mid-way."""
    bits, sym = case["bits"], case["sym"]
    xs = [G.arr(k) for k in case["xs"]]
    qm, quiet = _deferred_manager(bits, sym), _deferred_manager(bits, sym)
    mn, mx, stats = 0, 0, []
    for x in xs:
        xa = np.maximum(x, 0) if act == "relu" else x
        xt = torch.from_numpy(x).to(DEV)
        y = qm.quantize(xt, act=act) if act else qm.quantize(xt)
        quiet.quantize(xt.clone(), act=act) if act else quiet.quantize(xt.clone())
        np.testing.assert_array_equal(y.cpu().numpy(), xa)
        assert qm._pending_records, "the call should have taken the deferred path"
        stats.append(O.collect_stats(xa))
        mn, mx = O.observe_minmax(xa, mn, mx)
        s, z = O.minmax_qparams(mn, mx, sym, 8)
        want = dict(scale=s, zero_point=float(z), min_val=mn, max_val=mx, qp=(s, z),
                    mean_abs_x=[t[0] for t in stats], mean_x=[t[1] for t in stats], std=[t[2] for t in stats])
        _assert_read_equal(_read(qm), want)
        assert not qm._pending_records
    if act is None:
        cal = case["calib"]
        assert (qm.observer.min_val, qm.observer.max_val) == (cal["min_val"], cal["max_val"])
        assert float(qm.scale) == cal["scale"] and float(qm.zero_point) == cal["zero_point"]
    sync_calibration(nn.ModuleList([quiet]))
    a, b = _read(qm), _read(quiet)
    assert a == b   # exact: same records, same fold, same replay


def test_each_attribute_alone_folds():
    """Any one of the reads (observer min/max, get_scale_zero_point, zero_point, a stat
    list) folds the pending calls; a write of scale lands after them."""
    g = torch.Generator(device=DEV).manual_seed(5)
    xs = [torch.randn(3, 1000, device=DEV, generator=g) * (i + 1) for i in range(2)]
    readers = [lambda q: q.observer.min_val, lambda q: q.observer.max_val,
               lambda q: q.observer.get_scale_zero_point(), lambda q: q.zero_point, lambda q: q.scale,
               lambda q: q.mean_abs_x, lambda q: q.std]
    for read in readers:
        qm = _deferred_manager(8, False)
        for x in xs:
            qm.quantize(x)
        read(qm)
        assert not qm._pending_records
        want = O.observe_minmax(xs[1].cpu().numpy(), *O.observe_minmax(xs[0].cpu().numpy()))
        assert (qm.observer.min_val, qm.observer.max_val) == want
    qm = _deferred_manager(8, True)
    qm.quantize(xs[0])
    qm.scale = 0.5   # the reference overwrites after the call: the write wins
    assert not qm._pending_records and qm.scale == 0.5
    qm.quantize(xs[1])   # ...and the next call overwrites the write
    want = O.minmax_qparams(*O.observe_minmax(xs[1].cpu().numpy(), *O.observe_minmax(xs[0].cpu().numpy())),
                            True, 8)
    assert float(qm.scale) == want[0]


def test_deferred_read_under_dist_group_raises():
    """With a dist_group the fold needs every rank's records: a read raises a clear error
    naming sync_calibration instead of running a collective on one rank."""
    qm = _deferred_manager(8, True)
    qm.dist_group = object()   # never used for a collective before the read raises
    x = torch.randn(4096, device=DEV)
    qm.quantize(x)
    for read in (lambda: qm.scale, lambda: qm.observer.min_val, lambda: qm.mean_abs_x):
        with pytest.raises(RuntimeError, match="sync_calibration"):
            read()
    assert qm._pending_records
    qm.dist_group = None
    assert qm.observer.max_val == O.observe_minmax(x.cpu().numpy())[1]   # single GPU again: folds
    assert not qm._pending_records


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


def _loader(n=5):
    g = torch.Generator().manual_seed(1)
    return [(torch.randint(0, 256, (4, 3, 32, 32), generator=g, dtype=torch.uint8), None) for _ in range(n)]


def _managers(model):
    return [qm for m in model for qm in (m.weight_quantizer, m.activation_quantizer)]


def test_calibrate_qat_model_reads_per_batch_equal_per_call_path():
    """calibrate_qat_model with a data_calib that records every manager's state after each
    batch: the default deferred mode gives the per-call path's records (which the goldens
    pin, test_gpu_parity.py::test_golden_manager_sequence), and the final state is
    bit-identical to a deferred run that read nothing."""
    def recording(log):
        def calib(model, loader, device):
            model.eval()
            for imgs, _ in loader:
                model(imgs.to(device).float() / 255.0)
                log.append([_read(qm) for qm in _managers(model)])
            model.train()
        return calib

    a = _model()
    b, c = copy.deepcopy(a), copy.deepcopy(a)
    la, lb = [], []
    calibrate_qat_model(a, _loader(), recording(la), DEV)                         # default: deferred
    calibrate_qat_model(b, _loader(), recording(lb), DEV, defer_observers=False)  # per call
    calibrate_qat_model(c, _loader(), data_calib, DEV)                            # deferred, no reads
    assert len(la) == len(lb) == 5
    for ra, rb in zip(la, lb):
        for x, y in zip(ra, rb):
            _assert_read_equal(x, y)
    for qa, qc in zip(_managers(a), _managers(c)):
        assert not qa._pending_records and not qc._pending_records
        assert _read(qa) == _read(qc)


@pytest.mark.parametrize("mode", ["queued", "async"])
def test_reads_with_queued_or_async_deferred_calls(mode, monkeypatch):
    """The opt-in K2m queue (VSIQ_OBSERVE_BATCH=1: calls observed in batches) and the
    side-stream observers (async_observers=True): a read mid-calibration flushes / joins
    first, so the records equal the per-call path's."""
    import vsiquantization_amd.observe_batch as OB

    def recording(log):
        def calib(model, loader, device):
            model.eval()
            for imgs, _ in loader:
                model(imgs.to(device).float() / 255.0)
                log.append([_read(qm) for qm in _managers(model)])
            model.train()
        return calib

    a = _model()
    b = copy.deepcopy(a)
    la, lb = [], []
    if mode == "queued":
        monkeypatch.setenv("VSIQ_OBSERVE_BATCH", "1")
        calibrate_qat_model(a, _loader(), recording(la), DEV)
        monkeypatch.delenv("VSIQ_OBSERVE_BATCH")
        assert OB.pending() == 0
    else:
        calibrate_qat_model(a, _loader(), recording(la), DEV, async_observers=True)
    calibrate_qat_model(b, _loader(), recording(lb), DEV, defer_observers=False)
    for ra, rb in zip(la, lb):
        for x, y in zip(ra, rb):
            _assert_read_equal(x, y)


def test_copy_and_pickle_mid_calibration_fold_their_own_records(tmp_path):
    """A deep copy (EMA / teacher) or a torch.save of a manager taken while its deferred
    calls are pending: each copy folds its own copied records (the observer re-links to
    its own manager), the original is untouched by the copy's reads."""
    g = torch.Generator(device=DEV).manual_seed(9)
    xs = [torch.randn(5, 777, device=DEV, generator=g) * (i + 1) for i in range(3)]
    qm = _deferred_manager(8, False)
    for x in xs[:2]:
        qm.quantize(x)
    cp = copy.deepcopy(qm)
    path = tmp_path / "qm.pt"
    torch.save(qm, path)
    ld = torch.load(path, weights_only=False)   # our own file, written just above
    assert cp.observer._defer_owner() is cp and ld.observer._defer_owner() is ld
    want2 = O.observe_minmax(xs[1].cpu().numpy(), *O.observe_minmax(xs[0].cpu().numpy()))
    for c in (cp, ld):
        assert (c.observer.min_val, c.observer.max_val) == want2
        assert not c._pending_records
    assert len(qm._pending_records) == 2   # the copies' reads did not fold the original
    qm.quantize(xs[2])
    want3 = O.observe_minmax(xs[2].cpu().numpy(), *want2)
    assert (qm.observer.min_val, qm.observer.max_val) == want3
    assert len(qm.mean_abs_x) == 3 and len(cp.mean_abs_x) == 2
