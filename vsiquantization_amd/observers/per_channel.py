"""PerChannelMinMaxObserver — build-defined per-channel MinMax.

The reference has only a per-tensor MinMaxObserver (observers/minmax.py:6-88).
Per channel is defined as the reference observer applied independently to each
out-channel slice W[c] (axis 0 of OIHW / [out, in] weights):

    s_c, z_c = MinMaxObserver(symmetric, num_bits).forward(W[c])

with one running (min_val, max_val) per channel (fresh observers start at 0/0,
minmax.py:28-29).  All of it is one launch of the K3 kernel; scale and zero
point come back as float64 [C] device tensors (no host sync).  CPU tensors (the
reference's classes run on them, observers/minmax.py:42-43) take the native host
loops, row by row (host.pc_observe_fq): the same bits as K3.
"""
from __future__ import annotations

import torch

from .. import _hip as H
from .. import host as _host
from ..fakequant import PerChannelObserveFQFn, per_channel_observe_fq, qden
from ..utils.registry import register_class
from .base import BaseObserver


@register_class
class PerChannelMinMaxObserver(BaseObserver):
    axis = 0

    def __init__(self, symmetric=True, num_bits=8, eps=1e-8):
        self.symmetric = symmetric
        self.eps = eps
        self.num_bits = num_bits
        self.run_min = None   # fp32 [C] device
        self.run_max = None
        self.scale = None     # f64 [C] from the last observe
        self.zero_point = None

    # ------------------------------------------------------------------ state
    @property
    def min_val(self):
        return None if self.run_min is None else self.run_min.to(torch.float64)

    @property
    def max_val(self):
        return None if self.run_max is None else self.run_max.to(torch.float64)

    def _state(self, x):
        C = x.shape[0] if x.dim() > 0 else 1
        if self.run_min is None or self.run_min.numel() != C or self.run_min.device != x.device:
            state = torch.zeros(2, C, dtype=torch.float32, device=x.device)   # one fill
            self.run_min, self.run_max = state[0], state[1]
        return self.run_min, self.run_max

    def reset(self):
        self.run_min = self.run_max = self.scale = self.zero_point = None

    def __getstate__(self):
        # the bound C++ op (_op) is a cache of this state: not picklable, and a copy must
        # not keep launching on the original's running min / max -- rebuilt on first use
        # (deepcopy, e.g. ModelEMA's of a model holding this observer, and torch.save)
        state = self.__dict__.copy()
        state.pop("_op", None)
        return state

    # ------------------------------------------------------------------ protocol
    def observe(self, x, want_row_stats=False):
        x = x if _host.is_host(x) else H.require_device_f32(x)
        mn, mx = self._state(x)
        fn = _host.pc_observe_fq if _host.is_host(x) else per_channel_observe_fq
        r = fn(x, symmetric=self.symmetric, qmin=0, qmax=0, obs_bits=self.num_bits, eps=self.eps,
               run_min=mn, run_max=mx, quantize=False, want_row_stats=want_row_stats)
        self.scale, self.zero_point = r["scale"], r["zp"]
        return r["row_stats"]

    def get_scale_zero_point(self):
        """(scale f64[C], zero_point f64[C]) on the device, from the running state."""
        if self.scale is None:
            raise RuntimeError("PerChannelMinMaxObserver: nothing observed yet")
        return self.scale, self.zero_point

    def forward(self, x):
        self.observe(x)
        return self.get_scale_zero_point()

    def observe_quantize(self, x, quantizer, want_row_stats=False):
        """Fused observe + fake quant of ``x`` with ``quantizer``'s integer range (one pass).

        Returns (y, row_stats | None); y carries the STE gradient."""
        # the training step's call (public-API C2 step): straight to a C++ op bound to this
        # observer's state and the quantizer's range, which checks x itself (None back: the
        # general path below); rebuilt when either running tensor or the range changes
        op = self.__dict__.get("_op")
        if (op is not None and not want_row_stats and op[0] is self.run_min and op[1] is self.run_max
                and op[2] == (self.symmetric, self.num_bits, self.eps, quantizer.qmin, quantizer.qmax)
                and H.torch_ext_enabled()):
            r = op[3](x)
            if r is not None:
                y, self.scale, self.zero_point = r
                return y, None
        if (not want_row_stats and H.torch_ext_enabled() and isinstance(x, torch.Tensor) and x.is_cuda
                and x.dtype == torch.float32 and x.requires_grad and x.is_contiguous() and torch.is_grad_enabled()):
            mn, mx = self._state(x)
            op = self._op = (mn, mx, (self.symmetric, self.num_bits, self.eps, quantizer.qmin, quantizer.qmax),
                             H.torch_ext().PcObserveFqOp(mn, mx, bool(self.symmetric), int(quantizer.qmin),
                                                         int(quantizer.qmax),
                                                         qden(self.symmetric, self.num_bits, self.eps),
                                                         float(self.eps)))
            r = op[3](x)
            if r is not None:
                y, self.scale, self.zero_point = r
                return y, None
        if _host.is_host(x):
            mn, mx = self._state(x)
            args = (self.symmetric, quantizer.qmin, quantizer.qmax, self.num_bits, self.eps, mn, mx)
            if x.requires_grad and torch.is_grad_enabled():
                y, s, z, rs = _host.PcObserveFQFn.apply(x, *args, want_row_stats)
                rs = rs if want_row_stats else None
            else:
                r = _host.pc_observe_fq(x, symmetric=args[0], qmin=args[1], qmax=args[2], obs_bits=args[3],
                                        eps=args[4], run_min=mn, run_max=mx, want_row_stats=want_row_stats)
                y, s, z, rs = r["y"], r["scale"], r["zp"], r["row_stats"]
            self.scale, self.zero_point = s, z
            return y, rs
        x = H.require_device_f32(x)
        mn, mx = self._state(x)
        if H.torch_ext_enabled():   # C++ op (_vsiq_torch.so): an autograd node when x needs one
            y, s, z, rs = H.torch_ext().pc_observe_fq(x, mn, mx, bool(self.symmetric), int(quantizer.qmin),
                                                      int(quantizer.qmax), qden(self.symmetric, self.num_bits, self.eps),
                                                      float(self.eps), bool(want_row_stats))
            rs = rs if want_row_stats else None
        elif x.requires_grad and torch.is_grad_enabled():   # VSIQ_TORCH_EXT=0: the Python Function over ctypes
            y, s, z, rs = PerChannelObserveFQFn.apply(x, self.symmetric, quantizer.qmin, quantizer.qmax,
                                                      self.num_bits, self.eps, mn, mx, want_row_stats)
            rs = rs if want_row_stats else None
        else:
            r = per_channel_observe_fq(x, symmetric=self.symmetric, qmin=quantizer.qmin,
                                       qmax=quantizer.qmax, obs_bits=self.num_bits, eps=self.eps,
                                       run_min=mn, run_max=mx, want_row_stats=want_row_stats)
            y, s, z, rs = r["y"], r["scale"], r["zp"], r["row_stats"]
        self.scale, self.zero_point = s, z
        return y, rs

    def __repr__(self):
        return (f"PerChannelMinMaxObserver(symmetric={self.symmetric}, num_bits={self.num_bits}, "
                f"eps={self.eps}, axis=0)")
