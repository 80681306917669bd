"""Queued deferred observer calls (K2m, csrc/k_flat.hip).

In deferred calibration (``QuantizationManager.dist_defer``, the default of
``calibrate_qat_model``) an observer call only writes partial records that nothing reads
before ``sync_calibration`` (utils/quantize_manager.py:4-31 -> minmax.py:42-43 +
quantization_manager.py:66-68 per layer and batch).  So instead of one K2p launch per
layer, the call is queued -- the tensor is kept alive, its slot allocated -- and the
queue is observed in ONE multi-tensor launch (records bit-identical to per-call K2p)
when it holds 32 calls or ``VSIQ_OBSERVE_BATCH_BYTES`` of tensors (default 4 GiB of
the 288 GB HBM), when a call comes from another stream, and before anything reads the
records (``flush``; ``distributed.sync_calibration`` calls it).

OPT-IN (``VSIQ_OBSERVE_BATCH=1``): a queued tensor is the one the manager hands back to
the model, and it must not be modified in place before the flush (its version counter is
checked and a change raises; a write through ``.data`` is not seen).  By default every
deferred call is observed at once: a fused layer's call in one pass that also writes
the activation (K2o, ``fakequant.observe_parts_out``), any other call by K2p.
"""
from __future__ import annotations

import os

import torch

MAX_CALLS = 32


def enabled() -> bool:
    return os.environ.get("VSIQ_OBSERVE_BATCH", "0") == "1"


def _budget() -> int:
    return int(os.environ.get("VSIQ_OBSERVE_BATCH_BYTES", str(4 << 30)))


class _Queue:
    __slots__ = ("stream", "items", "bytes")

    def __init__(self):
        self.stream = None
        self.items = []    # (x, act, slot, version)
        self.bytes = 0


_QUEUES = {}


def add(x: torch.Tensor, act, slot: torch.Tensor):
    """Queue a deferred observer call of act(x) into ``slot``."""
    dev = x.device
    st = torch.cuda.current_stream(dev)
    q = _QUEUES.get(dev)
    if q is None:
        q = _QUEUES[dev] = _Queue()
    if q.items and q.stream != st:
        _flush(q)
    q.stream = st
    q.items.append((x, act, slot, x._version))
    q.bytes += x.numel() * x.element_size()
    if len(q.items) >= MAX_CALLS or q.bytes >= _budget():
        _flush(q)


def _flush(q: _Queue):
    from .fakequant import observe_parts_multi
    items, q.items, q.bytes = q.items, [], 0
    if not items:
        return
    changed = [it for it in items if it[0]._version != it[3]]
    ok = [it for it in items if it[0]._version == it[3]]
    with torch.cuda.stream(q.stream):
        for act in dict.fromkeys(a for _, a, _, _ in ok):
            sel = [(x, s) for x, a, s, _ in ok if a == act]
            observe_parts_multi([x for x, _ in sel], [s for _, s in sel], act=act)
        for x, _, _, _ in ok:   # x may come from another stream's pool: keep it until K2m ran
            x.record_stream(q.stream)
        for _, _, slot, _ in changed:   # record count 0: a later fold reads nothing from it
            slot.zero_()
    if changed:
        raise RuntimeError(f"{len(changed)} tensor(s) queued for a deferred observer were modified in place "
                           "before the observer ran (their calls recorded nothing); unset "
                           "VSIQ_OBSERVE_BATCH to observe each call at once")


def flush(device=None):
    """Observe every queued call (of ``device``, or of all devices) now; the current stream
    of each device then waits for its queue's launches (a later fold reads the records)."""
    for dev, q in list(_QUEUES.items()):
        if device is None or torch.device(device) == dev:
            st = q.stream
            _flush(q)
            if st is not None and st != torch.cuda.current_stream(dev):
                torch.cuda.current_stream(dev).wait_stream(st)


def pending(device=None) -> int:
    return sum(len(q.items) for dev, q in _QUEUES.items() if device is None or torch.device(device) == dev)
