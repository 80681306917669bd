"""MinMaxObserver on MI355X (reference: observers/minmax.py:6-88).

Same registry name, constructor ``(symmetric=True, num_bits=8, eps=1e-8)``,
attributes (``symmetric, eps, num_bits, min_val, max_val``) and methods
(``observe``, ``get_scale_zero_point``, ``forward``).

The running ``(min_val, max_val)`` state lives on the device as fp32[2] and is
updated by one pass of the K2 kernel per ``observe`` (the reference runs two
full reductions and two ``.item()`` syncs, minmax.py:42-43).  fp32 state is
exact: every value it can hold is an element of an fp32 tensor or the initial 0.
``min_val``/``max_val`` read it back lazily (one sync), returning the int ``0``
the reference starts with until a strictly smaller/larger value arrives.

A CPU tensor takes the same single pass in native host code (host.py; the state is then
a CPU fp32[2]).

``get_scale_zero_point``/``forward`` keep the reference's host semantics (Python
float scale, int zero point, ValueError/OverflowError from ``round`` on a
non-finite value).  ``observe_device`` is the sync-free path used by
QuantizationManager: it returns the f64 qparams record computed on the device.
"""
from __future__ import annotations

import torch

from .. import _hip as H
from .. import host
from ..fakequant import observe_tensor
from ..utils.registry import register_class
from .base import BaseObserver


def _host_number(v: float):
    # 0 can only mean "never updated" (strict compares, minmax.py:44-47): reference keeps int 0
    return 0 if v == 0.0 else v


@register_class
class MinMaxObserver(BaseObserver):
    # weakref to the QuantizationManager whose deferred calibration calls (not folded yet)
    # hold this observer's later updates: any read or update folds them first
    _defer_owner = None

    def __init__(self, symmetric=True, num_bits=8, eps=1e-8):
        self.symmetric = symmetric
        self.eps = eps
        self.num_bits = num_bits
        self._state = None          # device fp32[2]: running (min_val, max_val)
        self._host = [0, 0]         # host mirror, valid when not self._dirty
        self._dirty = False
        self._obs_stream = None     # side stream with pending updates (async calibration)

    def __getstate__(self):
        # the owner link is a weakref (not picklable) to the manager this observer belongs
        # to; a copy's manager re-links its own copy (QuantizationManager.__setstate__)
        state = self.__dict__.copy()
        state.pop("_defer_owner", None)
        return state

    # ------------------------------------------------------------------ state
    def _join(self):
        """Make the current stream wait for updates queued on a side stream."""
        if self._obs_stream is not None:
            if self._state is not None:
                torch.cuda.current_stream(self._state.device).wait_stream(self._obs_stream)
            self._obs_stream = None

    def _fold_owner(self):
        owner = self._defer_owner()
        if owner is None:
            self._defer_owner = None
        else:
            owner._fold_pending()

    def _sync(self):
        if self._defer_owner is not None:
            self._fold_owner()
        self._join()
        if self._dirty:
            mn, mx = self._state.tolist()
            self._host = [_host_number(mn), _host_number(mx)]
            self._dirty = False

    @property
    def min_val(self):
        self._sync()
        return self._host[0]

    @min_val.setter
    def min_val(self, v):
        self._set(0, v)

    @property
    def max_val(self):
        self._sync()
        return self._host[1]

    @max_val.setter
    def max_val(self, v):
        self._set(1, v)

    def _set(self, i, v):
        self._sync()   # joins a pending side stream first
        self._host[i] = v
        if self._state is not None:
            self._state[i] = 0.0 if v is None else float(v)

    def device_state(self, device) -> torch.Tensor:
        """fp32[2] running (min, max) on ``device`` (created from the host values)."""
        device = torch.device(device)
        if self._state is None or self._state.device != device:
            self._sync()
            vals = [0.0 if v is None else float(v) for v in self._host]
            self._state = torch.tensor(vals, dtype=torch.float32, device=device)
        return self._state

    def reset(self):
        if self._defer_owner is not None:
            self._fold_owner()
        self._state = None
        self._host = [0, 0]
        self._dirty = False

    # ------------------------------------------------------------------ protocol
    def observe_device(self, x, want_stats=True, want_qp=True, act=None):
        """One K2 pass: update the running state, return (qp f64[4], stats f64[10]) on x.device.
        ``act``: observe act(x) (fused ReLU/SiLU, K5) without materializing it."""
        if self._defer_owner is not None:
            self._fold_owner()
        if host.is_host(x):   # CPU tensor: the native host pass (host.py), CPU fp32[2] state
            dev = x.device
        else:
            dev = H.require_device_f32(x).device
            if self._obs_stream is not None and self._obs_stream != torch.cuda.current_stream(dev):
                self._join()
        state = self.device_state(dev)
        qp, st = observe_tensor(x, symmetric=self.symmetric, num_bits=self.num_bits, eps=self.eps,
                                run_minmax=state, want_qp=want_qp, want_stats=want_stats, act=act)
        self._dirty = True
        return qp, st

    def observe(self, x):
        """Update min/max from ``x`` (minmax.py:32-47)."""
        self.observe_device(x, want_stats=False, want_qp=False)

    def get_scale_zero_point(self):
        """Host float64 qparams (minmax.py:49-74)."""
        mn, mx = self.min_val, self.max_val
        if self.symmetric:
            max_abs = max(abs(mn), abs(mx))
            scale = max_abs / (2 ** (self.num_bits - 1) - 1 + self.eps)
            zero_point = 0
        else:
            scale = (mx - mn) / (2 ** self.num_bits - 1 + self.eps)
            zero_point = round(-mn / (scale + self.eps))
        return scale, zero_point

    def forward(self, x):
        """observe + get_scale_zero_point (minmax.py:76-88); one device->host read."""
        self.observe(x)
        return self.get_scale_zero_point()

    def __repr__(self):
        return (f"MinMaxObserver(symmetric={self.symmetric}, num_bits={self.num_bits}, "
                f"eps={self.eps})")


@register_class
class LSQObserver(MinMaxObserver):
    """The observer name README.md:131 advertises but the reference never registers
    (SURVEY §0.1).  In the reference's QAT flow an observer only feeds the calibration
    statistics; the LSQ step size itself is initialised from mean(|x|)
    (QuantizationManager.init_scaling_factor_for_learning, qm.py:105-112), so
    LSQObserver is MinMaxObserver's K2 pass under the README's name."""
