"""Host logic of the lazy fold of deferred calibration calls (quantization_manager.py
_defer_begin / _fold_pending / __getattr__ / __setattr__, minmax.py _defer_owner), without
a GPU: the device fold (distributed.fold_slots) is replaced by a stand-in that returns
given stats records, so what is checked is when the fold runs and that the replay gives
the reference's per-call state (observers/minmax.py:42-47, quantization_manager.py:55-71).
The kernels' records themselves are pinned on the GPU (tests/test_gpu_calib_reads.py)."""
import copy
import pickle

import pytest
import torch

import vsiquantization_amd as V
from vsiquantization_amd import _hip as H
from vsiquantization_amd import distributed as D
from oracle import fakequant_np as O


def _record(mn, mx, nan=0, mean_abs=1.0, mean=0.0, std=1.0):
    r = torch.zeros(H.ST_LEN, dtype=torch.float64)
    r[H.ST_MIN], r[H.ST_MAX], r[H.ST_NAN] = mn, mx, nan
    r[H.ST_MEANABS], r[H.ST_MEAN], r[H.ST_STD] = mean_abs, mean, std
    return r


@pytest.fixture
def fake_fold(monkeypatch):
    """Pending "slots" are the stats records themselves; the fold stacks them."""
    calls = []

    def fold(slots):
        calls.append(len(slots))
        return torch.stack(slots)
    monkeypatch.setattr(D, "fold_slots", fold)
    return calls


def _manager(sym=False):
    qm = V.QuantizationManager("UniformQuantizer", "MinMaxObserver", 8, sym, True)
    qm.is_observer_qparam, qm.is_learning_scale, qm.is_quantize = True, False, False
    return qm


def _call(qm, rec):
    """What _collect_distributed / _observe_deferred_act do for one deferred call."""
    if not qm._pending_records:
        qm._defer_begin()
    qm._pending_records.append(rec)


CALLS = [(-0.5, 1.25), (-2.0, 0.75), (float("nan"), float("nan"), 1), (-1.0, 3.5)]


def _replayed(k, sym=False):
    mn, mx = 0, 0
    for c in CALLS[:k]:
        if len(c) == 3:   # a NaN call changes nothing (minmax.py:44-47)
            continue
        mn = c[0] if c[0] < mn else mn
        mx = c[1] if c[1] > mx else mx
    return (mn, mx), O.minmax_qparams(mn, mx, sym, 8)


def test_each_read_sees_the_calls_so_far(fake_fold):
    qm = _manager()
    for k, c in enumerate(CALLS, 1):
        _call(qm, _record(*c, mean_abs=float(k)))
        assert "scale" not in qm.__dict__ and qm.observer._defer_owner() is qm
        (mn, mx), (s, z) = _replayed(k)
        assert (qm.observer.min_val, qm.observer.max_val) == (mn, mx)
        assert (qm.scale, qm.zero_point) == (s, z)
        assert qm.mean_abs_x == [float(j) for j in range(1, k + 1)]
        assert not qm._pending_records and qm.observer._defer_owner is None
    assert fake_fold == [1, 1, 1, 1]


def test_no_read_folds_once_and_ends_in_the_same_state(fake_fold):
    a, b = _manager(), _manager()
    for k, c in enumerate(CALLS, 1):
        _call(a, _record(*c, mean_abs=float(k)))
        _call(b, _record(*c, mean_abs=float(k)))
        a.scale   # noqa: B018  (a read folds)
    D.sync_calibration(torch.nn.ModuleList([b]))
    assert fake_fold == [1, 1, 1, 1, 4]
    for qm in (a, b):
        assert (qm.observer.min_val, qm.observer.max_val) == _replayed(4)[0]
        assert (qm.scale, qm.zero_point) == _replayed(4)[1]
        assert qm.mean_abs_x == [1.0, 2.0, 3.0, 4.0]


def test_write_of_scale_lands_after_the_pending_calls(fake_fold):
    qm = _manager(sym=True)
    _call(qm, _record(-1.0, 2.0))
    qm.scale = 0.125
    assert not qm._pending_records and qm.scale == 0.125
    _call(qm, _record(-3.0, 1.0))
    assert qm.scale == O.minmax_qparams(-3.0, 2.0, True, 8)[0]


def test_observer_reads_and_updates_fold_first(fake_fold):
    qm = _manager()
    _call(qm, _record(-1.0, 2.0))
    assert qm.observer.get_scale_zero_point() == O.minmax_qparams(-1.0, 2.0, False, 8)
    _call(qm, _record(-4.0, 2.0))
    qm.observer.observe(torch.tensor([5.0, -0.25]))   # host observe after the pending call
    assert (qm.observer.min_val, qm.observer.max_val) == (-4.0, 5.0)
    _call(qm, _record(-8.0, 1.0))
    qm.observer.reset()
    assert not qm._pending_records and (qm.observer.min_val, qm.observer.max_val) == (0, 0)


def test_read_under_a_process_group_raises(fake_fold):
    qm = _manager()
    qm.dist_group = object()
    _call(qm, _record(-1.0, 2.0))
    for read in (lambda: qm.scale, lambda: qm.zero_point, lambda: qm.observer.max_val, lambda: qm.std):
        with pytest.raises(RuntimeError, match="sync_calibration"):
            read()
    assert fake_fold == [] and len(qm._pending_records) == 1


def test_copies_fold_their_own_records(fake_fold):
    qm = _manager()
    _call(qm, _record(-1.0, 2.0))
    _call(qm, _record(-3.0, 0.5))
    for cp in (copy.deepcopy(qm), pickle.loads(pickle.dumps(qm))):
        assert cp.observer._defer_owner() is cp
        assert (cp.observer.min_val, cp.observer.max_val) == (-3.0, 2.0)
        assert len(qm._pending_records) == 2
    assert (qm.observer.min_val, qm.observer.max_val) == (-3.0, 2.0)


def test_hasattr_under_a_process_group_is_false(fake_fold):
    """hasattr(qm, "scale") during a deferred multi-GPU calibration answers False (the read
    raises DeferredSyncError, a RuntimeError that is also an AttributeError) and folds
    nothing."""
    from vsiquantization_amd.quantizers.quantization_manager import DeferredSyncError
    qm = _manager()
    qm.dist_group = object()
    _call(qm, _record(-1.0, 2.0))
    assert not hasattr(qm, "scale") and not hasattr(qm, "zero_point")
    with pytest.raises(DeferredSyncError, match="sync_calibration"):
        qm.scale
    assert fake_fold == [] and len(qm._pending_records) == 1


def test_failing_replay_keeps_the_calls(monkeypatch, fake_fold):
    """A fold whose replay raises leaves the manager as it was: the calls stay pending and a
    later read (once the replay works) gives the reference's state."""
    qm = _manager()
    for c in CALLS:
        _call(qm, _record(*c))

    def boom(*a, **k):
        raise RuntimeError("replay failed")
    monkeypatch.setattr(D, "replay_minmax", boom)
    with pytest.raises(RuntimeError, match="replay failed"):
        qm.scale
    assert len(qm._pending_records) == len(CALLS) and qm._calib_init == (0, 0)
    monkeypatch.undo()
    monkeypatch.setattr(D, "fold_slots", lambda slots: torch.stack(slots))
    assert (qm.observer.min_val, qm.observer.max_val) == _replayed(len(CALLS))[0]
    assert qm._pending_records == []
