"""QuantizationManager (reference: quantizers/quantization_manager.py:10-145).

nn.Module owning one quantizer and one observer, built by registry name
(qm.py:41-42), with the reference's mode flags, attributes and methods:
``quantizer, observer, scale, zero_point, is_observer_qparam, is_learning_scale,
is_quantize, is_symmetric (hard-coded True, qm.py:50), bits_width, mean_abs_x,
mean_x, std``; ``collect_qparameter, quantize, make_learn_qparameter,
init_scaling_factor_for_learning, winsorized_mean``.

MI355X differences (behaviour-preserving):
* With this package's observers, ``collect_qparameter`` is sync-free: the observer
  kernel writes the f64 qparams record on the device and ``self.scale`` /
  ``self.zero_point`` become 0-dim device tensors that the quantizer kernel reads
  by pointer (the reference performs five ``.item()`` syncs per call, qm.py:66-69).
* ``mean_abs_x / mean_x / std`` are kept as device records and materialised into
  the reference's Python lists of floats on first read (one sync).
* Per-channel observer + per-channel quantizer in observe+quantize mode run as ONE
  fused kernel (observe, f64 qparams and fake quant in one read of ``x``).
"""
from __future__ import annotations

import itertools
import warnings
import weakref

import numpy as np
import torch
import torch.nn as nn

from .. import _hip as H
from .. import observe_batch
from ..fakequant import activation as _activation
from ..fakequant import (observe_parts, observe_tensor, part_slot_doubles,
                         stats_from_row_sums)
from ..observers.minmax import MinMaxObserver
from ..observers.per_channel import PerChannelMinMaxObserver
from ..utils.registry import CLASS_REGISTRY
from .per_channel import PerChannelUniformQuantizer

_STAT_NAMES = ("mean_abs_x", "mean_x", "std")


def _as_f32(t: torch.Tensor) -> torch.Tensor:
    """f64 stats -> the fp32 values the reference's lists hold (quantization_manager.py:66-68
    append torch.mean / torch.std of an fp32 tensor, .item()-ed: fp32 values), kept as f64.
    Under a mean reference mean|x| / mean are torch's bits already (K11) and the f64 std
    rounds to torch's fp32 std (its two-pass f64 sum about the fp32 mean, rounded once)."""
    return t.to(torch.float32).to(torch.float64)
_QP_ATTRS = ("scale", "zero_point")

# Calibration-time observer streams: an observe-only call (is_quantize False) has no
# consumer until calibration ends, so its K2 pass is queued on a side stream and the
# model's next layers do not wait for it (its reduction tail overlaps their work).
# Managers are spread round-robin over a small per-device pool; each manager always
# uses the same stream, so its own running state stays stream-ordered.
# Per-call observe+quantize in one call (fakequant.observe_fake_quant): K8 (one launch,
# one workgroup holds the tensor) up to 16384 elements, K9 (K2p records + a fake-quant
# launch folding them in every workgroup, no arrival chain) up to this many.
_OBSERVE_FQ_MAX = 1 << 18

_OBS_POOL = 4
_OBS_STREAMS = {}
_MGR_IDS = itertools.count()


class DeferredSyncError(RuntimeError, AttributeError):
    """A read of scale / zero_point that needs every rank's deferred records (call
    sync_calibration first).  Also an AttributeError, so hasattr(manager, "scale") answers
    False instead of raising; the other reads (stat lists, observer state) raise the plain
    RuntimeError, since an AttributeError from a property would be replaced by a bare
    "no attribute" one."""


class _NeedsAllRanks(RuntimeError):
    pass


def _observer_stream(device, idx):
    pool = _OBS_STREAMS.get(device)
    if pool is None:
        pool = _OBS_STREAMS[device] = [torch.cuda.Stream(device=device) for _ in range(_OBS_POOL)]
    return pool[idx % len(pool)]


class _StatList:
    """Property backing one of mean_abs_x / mean_x / std (a Python list of floats)."""

    def __init__(self, idx):
        self.idx = idx

    def __get__(self, obj, objtype=None):
        if obj is None:
            return self
        obj._fold_pending()
        obj._materialize_stats()
        return obj._host_stats[self.idx]

    def __set__(self, obj, value):
        obj._fold_pending()
        obj._materialize_stats()
        obj._host_stats[self.idx] = value


class QuantizationManager(nn.Module):
    mean_abs_x = _StatList(0)
    mean_x = _StatList(1)
    std = _StatList(2)

    def __init__(self, quantizer_name: str, observer_name: str, bits_width: int, is_symmetric: bool,
                 is_learning_scale: bool = True) -> None:
        super().__init__()
        self.quantizer = CLASS_REGISTRY[quantizer_name](bits_width, is_symmetric)
        self.observer = CLASS_REGISTRY[observer_name](is_symmetric)
        self.is_learning_scale = is_learning_scale
        self.bits_width = bits_width
        self.scale = 1
        self.zero_point = 0
        self.is_observer_qparam = True
        self.is_quantize = True
        self.is_symmetric = True   # reference quirk (qm.py:50): observer/quantizer keep their own flag
        self._dev_stats = []       # pending device records f64[3] (mean|x|, mean, std)
        self._host_stats = [[], [], []]
        # multi-GPU observer (vsiquantization_amd.distributed): process group, deferred mode
        self.dist_group = None
        self.dist_defer = False
        self._pending_records = []   # deferred: per-call K2p partial-record slots (f64)
        self._calib_init = None
        # observe-only calls queued on a side stream (see _observer_stream).  Off by
        # default (then scale / zero_point are plain stream-ordered device tensors);
        # calibrate_qat_model turns it on for the calibration run and joins at the end.
        self.async_observer = False
        self._obs_id = next(_MGR_IDS)
        self._side = None            # side stream with this manager's pending records
        self.mean_abs_x = []
        self.mean_x = []
        self.std = []
        # (W, threads) of the reference CPU layout of the fused SiLU (vsiq_common.cuh
        # silu_lay) this manager's qparams were observed / learned with: recorded at the
        # first SiLU call, used for every later one, saved in the state_dict
        # ("<prefix>silu_layout", only once recorded)
        self.silu_layout = None

    # ------------------------------------------------------------------ SiLU layout
    def _silu_act(self, act):
        """act, with "silu" bound to this manager's recorded layout (H.SiluAct)."""
        if act != "silu" or isinstance(act, H.SiluAct):
            return act
        cur = H.silu_reference()
        lay = self.__dict__.get("silu_layout")
        if lay is None:
            self.silu_layout = lay = tuple(cur)
        elif tuple(cur) != tuple(lay) and not self.__dict__.get("_silu_warned"):
            self._silu_warned = True
            warnings.warn(f"QuantizationManager: SiLU reference layout (W, threads) {tuple(lay)} recorded with "
                          f"these qparams differs from this process's {tuple(cur)}; the recorded one is used "
                          f"(torch's CPU F.silu bits depend on it; H.set_silu_reference pins another)",
                          RuntimeWarning, stacklevel=3)
        return H.SiluAct(*lay)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        super()._save_to_state_dict(destination, prefix, keep_vars)
        lay = self.__dict__.get("silu_layout")
        if lay is not None:
            destination[prefix + "silu_layout"] = torch.tensor(lay, dtype=torch.int64)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        key = prefix + "silu_layout"
        if key in state_dict:
            self.silu_layout = tuple(int(v) for v in state_dict[key].reshape(-1).tolist())
            self._silu_warned = False
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)
        if key in unexpected_keys:
            unexpected_keys.remove(key)

    # ------------------------------------------------------------------ deferred calls
    # While deferred calibration calls are pending (dist_defer: K2p / K2o records, folded
    # by distributed.sync_calibration), scale / zero_point are out of __dict__, so a read
    # lands in __getattr__ and folds this manager's calls first: every read during
    # calibration sees what the reference holds after the calls so far (qm.py:55-71,
    # minmax.py:42-47).  The stat lists and the observer's min/max fold the same way.
    def __getattr__(self, name):
        if name in _QP_ATTRS and self.__dict__.get("_pending_records"):
            try:
                self._fold_pending()
            except _NeedsAllRanks as e:   # also an AttributeError here (hasattr)
                raise DeferredSyncError(str(e)) from None
            return getattr(self, name)
        return nn.Module.__getattr__(self, name)

    def __setattr__(self, name, value):
        if name in _QP_ATTRS and self.__dict__.get("_pending_records"):
            self._fold_pending()   # the calls before this write happened first
        nn.Module.__setattr__(self, name, value)

    def __setstate__(self, state):
        # a deep copy / unpickle taken while deferred calls were pending: the copied
        # observer folds into THIS manager's copied records, never the original's
        super().__setstate__(state)
        if self.__dict__.get("_pending_records") and isinstance(self.__dict__.get("observer"), MinMaxObserver):
            self.observer._defer_owner = weakref.ref(self)

    def _defer_begin(self):
        """First deferred call since the last fold: keep the running state the replay
        starts from, and route reads of the qparams / observer state to _fold_pending."""
        obs = self.observer
        self._calib_init = (obs.min_val, obs.max_val)
        d = self.__dict__
        for k in _QP_ATTRS:
            d.pop(k, None)
        if isinstance(obs, MinMaxObserver):
            obs._defer_owner = weakref.ref(self)

    def _fold_pending(self):
        """Fold this manager's pending deferred calls now (single GPU; one fold launch and
        one device->host read), exactly as sync_calibration would at the end.  Under a
        dist_group the fold needs every rank's records: RuntimeError."""
        pend = self.__dict__.get("_pending_records")
        if not pend:
            return
        if self.dist_group is not None:
            raise _NeedsAllRanks("QuantizationManager: scale / zero_point / mean_abs_x / observer state read during "
                               "a deferred multi-GPU calibration; these need every rank's records -- call "
                               "vsiquantization_amd.distributed.sync_calibration(model) on every rank first")
        from ..distributed import fold_slots
        observe_batch.flush()
        self._join()
        self._apply_synced_records(fold_slots(pend).cpu())

    # ------------------------------------------------------------------ side stream
    def _join(self):
        """Make the current stream wait for this manager's observer work on its side stream
        (before any consumer of the scale / zero point / stats records / observer state)."""
        side = self.__dict__.get("_side")
        if side is not None:
            self.__dict__["_side"] = None
            torch.cuda.current_stream(side.device).wait_stream(side)
            obs = self.__dict__.get("observer")
            if isinstance(obs, MinMaxObserver):
                obs._join()

    # ------------------------------------------------------------------ stats records
    def _materialize_stats(self):
        self._join()
        pend = self.__dict__.get("_dev_stats")
        if pend:
            rows = _as_f32(torch.stack(pend).cpu()).tolist()
            self.__dict__["_dev_stats"] = []
            for r in rows:
                for i in range(3):
                    self._host_stats[i].append(r[i])

    def _record_stats(self, st3: torch.Tensor, x=None, act=None):
        """st3: (mean|x|, mean, std) of this call.  With a mean reference set
        (H.set_mean_reference) and the call's tensor given, mean|x| / mean / std are replaced
        by torch CPU's bits for that host layout (K11 and its std pass,
        fakequant.torch_stats; CPU tensors: the means, the host record's std)."""
        if x is not None and H.mean_reference() is not None and self.dist_group is None:
            ex = self._exact_stats(x, act)
            st3 = st3.clone()
            if ex.device.type == "cpu":   # CPU tensor: the means; the host record's std stays
                st3[:2] = ex[:2].to(st3.device)
            else:
                st3.copy_(ex)
        self._dev_stats.append(st3)

    @staticmethod
    def _exact_stats(x, act):
        """f64[3] mean|x| / mean / std of act(x) as the reference host's torch records them
        (fakequant.torch_stats: K11 and its std pass; CPU tensors: the means, std NaN)."""
        from ..fakequant import torch_stats
        return torch_stats(x.detach(), act=act)

    # ------------------------------------------------------------------ observe
    def _device_observer(self, x) -> bool:
        return (isinstance(x, torch.Tensor) and x.device.type == "cuda"
                and isinstance(self.observer, (MinMaxObserver, PerChannelMinMaxObserver)))

    def collect_qparameter(self, x, act=None):
        """Observe ``x`` (or act(x), K5) and refresh scale/zero_point when calibrating
        (qm.py:55-71)."""
        if self.is_learning_scale or not self.is_observer_qparam:
            return
        if act is not None:
            act = self._silu_act(act)
        if isinstance(x, torch.Tensor):
            self._x_device = x.device   # where this layer's tensors live (_home_device)
        if act is not None and not self._act_fusable(x):
            x, act = _activation(x, act), None
        if (self.async_observer and not self.is_quantize and self._device_observer(x)
                and not isinstance(self.observer, PerChannelMinMaxObserver)):
            # observe-only: queue on this manager's side stream, do not wait for it
            main = torch.cuda.current_stream(x.device)
            side = _observer_stream(x.device, self._obs_id)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self._observe_device(x, act)
            x.record_stream(side)
            self._side = side
            self.observer._obs_stream = side
            return
        self._join()
        self._observe_device(x, act) if self._device_observer(x) else self._observe_host(x)

    def _observe_device(self, x, act):
        if isinstance(self.observer, PerChannelMinMaxObserver):
            rs = self.observer.observe(x, want_row_stats=True)
            self._record_stats(stats_from_row_sums(rs, x.numel()), x)
            self.scale, self.zero_point = self.observer.get_scale_zero_point()
        elif self.dist_group is not None or self.dist_defer:
            self._collect_distributed(x, act)
        else:
            qp, st = self.observer.observe_device(x, act=act)
            self._record_stats(st[H.ST_MEANABS:H.ST_STD + 1], x, act)
            self.scale, self.zero_point = qp[H.QP_SCALE], qp[H.QP_ZP]

    def _observe_host(self, x):
        from .. import host
        obs = self.observer
        if host.is_host(x) and isinstance(obs, MinMaxObserver) and not isinstance(obs, PerChannelMinMaxObserver):
            # CPU tensor, this package's observer: one native host pass (host.py) for the
            # running state and the mean|x| / mean / std record; qparams as the
            # reference's host numbers (minmax.py:49-74)
            _, st = obs.observe_device(x.detach(), want_qp=False)
            self._record_stats(st[H.ST_MEANABS:H.ST_STD + 1], x)
            self.scale, self.zero_point = obs.get_scale_zero_point()
            return
        # third-party observer: the reference's host path
        xd = x.detach()
        self._materialize_stats()
        self._host_stats[0].append(torch.mean(torch.abs(xd)).cpu().item())
        self._host_stats[1].append(torch.mean(xd).cpu().item())
        self._host_stats[2].append(torch.std(xd).cpu().item())
        self.scale, self.zero_point = self.observer.forward(x)

    # ------------------------------------------------------------------ multi-GPU observer
    def _collect_distributed(self, x, act=None):
        from ..distributed import gather_finalize
        obs = self.observer
        if self.dist_defer:
            # deferred (calibration): K2p partial records only -- no fold, no running
            # update, no collective -- until sync_calibration folds every call at once
            if self.is_quantize:
                raise RuntimeError("deferred observer sync (dist_defer) needs is_quantize=False "
                                   "(calibration); use per-call mode to quantize while observing")
            if not self._pending_records:
                self._defer_begin()
            slot = torch.empty(part_slot_doubles(x.numel()), dtype=torch.float64, device=x.device)
            if observe_batch.enabled():   # opt-in queue: one K2m launch per up to 32 calls
                observe_batch.add(x, act, slot)
                self._pending_records.append(slot)
            else:
                self._pending_records.append(observe_parts(x, out=slot, act=act))
            self._defer_exact(x, act)
            return
        _, st = observe_tensor(x, symmetric=obs.symmetric, num_bits=obs.num_bits, eps=obs.eps,
                               run_minmax=None, want_qp=False, want_stats=True, act=act)
        state = obs.device_state(x.device)
        st, qp = gather_finalize(st, state, symmetric=obs.symmetric, num_bits=obs.num_bits, eps=obs.eps,
                                 group=self.dist_group)
        obs._dirty = True
        self._record_stats(st[H.ST_MEANABS:H.ST_STD + 1])
        self.scale, self.zero_point = qp[H.QP_SCALE], qp[H.QP_ZP]

    def _defer_exact(self, x, act):
        """A deferred call under a mean reference: its exact means (K11) now, while x is
        alive; _apply_synced_records puts them in place of the records' means."""
        ex = self.__dict__.setdefault("_exact_pending", [])
        while len(ex) < len(self._pending_records) - 1:
            ex.append(None)
        ex.append(self._exact_stats(x, act) if (H.mean_reference() is not None and self.dist_group is None)
                  else None)

    def _apply_synced_records(self, recs):
        """recs: CPU f64 [k, ST_LEN], already all-reduced; replay the running state.  Every
        value is computed first; the pending records are dropped only when that worked
        (a failing replay leaves the manager as it was, its calls still pending)."""
        from ..distributed import replay_minmax
        mn, mx = self._calib_init
        exact = self.__dict__.get("_exact_pending") or []
        if any(e is not None for e in exact):
            recs = recs.clone()
            for i, e in enumerate(exact[:recs.shape[0]]):
                if e is not None:
                    m = e.cpu()
                    recs[i, H.ST_MEANABS] = float(m[0])
                    recs[i, H.ST_MEAN] = float(m[1])
                    if not torch.isnan(m[2]):
                        recs[i, H.ST_STD] = float(m[2])
        mn, mx = replay_minmax(mn, mx, recs[:, [H.ST_MIN, H.ST_MAX, H.ST_NAN]].tolist())
        cols = [_as_f32(recs[:, col]).tolist() for col in (H.ST_MEANABS, H.ST_MEAN, H.ST_STD)]
        # commit: no pending records from here on, so the writes below do not fold again
        d = self.__dict__
        d["_pending_records"] = []
        d.pop("_exact_pending", None)
        d["_calib_init"] = None
        obs = self.observer
        if isinstance(obs, MinMaxObserver):
            obs._defer_owner = None
        obs.min_val, obs.max_val = mn, mx
        self._materialize_stats()
        for i, col in enumerate(cols):
            self._host_stats[i].extend(col)
        self.scale, self.zero_point = obs.get_scale_zero_point()

    def _act_fusable(self, x) -> bool:
        """Can act(x) be fused into this manager's kernels (K5)?  Needs a CUDA tensor,
        this package's per-tensor quantizer and (when observing) per-tensor observer."""
        from .uniform import UniformQuantizer
        if not (isinstance(x, torch.Tensor) and x.device.type == "cuda"):
            return False
        if not isinstance(self.quantizer, UniformQuantizer) or isinstance(self.quantizer,
                                                                          PerChannelUniformQuantizer):
            return False
        observing = not self.is_learning_scale and self.is_observer_qparam
        return not observing or (isinstance(self.observer, MinMaxObserver)
                                 and not isinstance(self.observer, PerChannelMinMaxObserver))

    def quantize(self, x, act=None):
        """collect_qparameter, then fake-quantize when enabled (qm.py:73-90).

        ``act`` ("relu" / "silu"): the layer's activation, applied to ``x`` first; with
        this package's kernels it is fused into the observer and the fake quant (K5); a
        SiLU uses the reference layout recorded with this manager's qparams (silu_layout)."""
        if act is not None:
            act = self._silu_act(act)
        if self.is_quantize or self.is_learning_scale:
            self._join()
        if self.is_learning_scale and self.is_quantize:
            # training (learnable qparams): the branches below that observe need
            # `not is_learning_scale` and collect_qparameter returns at once, so this is
            # the same sequence without their checks (host time per call of a QAT step)
            if act is not None and not self._act_fusable(x):
                x, act = _activation(x, act), None
            d = self.__dict__.pop("_deferred_qparams", None)   # quantizers/deferred.py bundle
            if d is not None:
                from .deferred import deferred_learn
                q = self.quantizer
                gscale, zp, learn_zp = q.learn_args(x, d[1])
                if not isinstance(gscale, torch.Tensor) and learn_zp != 2:
                    return deferred_learn(x, d[0], zp, q.qmin, q.qmax, gscale, learn_zp, act)
            if act is None:
                return self.quantizer.quantize(x, self.scale, self.zero_point, True)
            return self.quantizer.quantize(x, self.scale, self.zero_point, True, act=act)
        if (act is not None and not self.is_quantize and self.dist_defer and not self.is_learning_scale
                and self.is_observer_qparam and self._act_fusable(x)
                and not (x.requires_grad and torch.is_grad_enabled())):
            return self._observe_deferred_act(x, act)
        if act is not None and not (self.is_quantize and self._act_fusable(x)):
            x, act = _activation(x, act), None
        if act is None and (self.is_quantize and not self.is_learning_scale and self.is_observer_qparam
                and isinstance(self.observer, PerChannelMinMaxObserver)
                and isinstance(self.quantizer, PerChannelUniformQuantizer) and self._device_observer(x)):
            # fused per-channel observe + quantize: one read, one write of x
            y, rs = self.observer.observe_quantize(x, self.quantizer, want_row_stats=True)
            self._record_stats(stats_from_row_sums(rs, x.numel()), x)
            self.scale, self.zero_point = self.observer.get_scale_zero_point()
            return y
        if act is None or self._act_fusable(x):
            y = self._observe_quantize_ranks(x, act)
            if y is None:
                y = self._observe_quantize_small(x, act)
            if y is not None:
                return y
        self.collect_qparameter(x, act)
        if self.is_quantize:
            if act is None:
                return self.quantizer.quantize(x, self.scale, self.zero_point, self.is_learning_scale)
            return self.quantizer.quantize(x, self.scale, self.zero_point, self.is_learning_scale,
                                           act=act)
        return x

    def _observe_deferred_act(self, x, act):
        """A fused layer's deferred calibration call (calibrate_qat_model's default mode):
        y = act(x), which the next layer consumes, and this call's K2p records of act(x) in
        ONE pass (K2o, fakequant.observe_parts_out).  Nothing is queued, so user code may
        modify y in place (ReLU(inplace=True), a residual +=) before calibration ends."""
        from ..fakequant import observe_parts_out, part_out_slot_doubles
        self._join()
        self._x_device = x.device
        if not self._pending_records:
            self._defer_begin()
        slot = torch.empty(part_out_slot_doubles(x.numel()), dtype=torch.float64, device=x.device)
        y, _ = observe_parts_out(x, act, out=slot)
        self._pending_records.append(slot)
        self._defer_exact(x, act)
        return y

    def _observe_quantize_ranks(self, x, act):
        """Multi-GPU per-call observe + quantize (dist_group set, not deferred): the local
        K2 pass, one all_gather of the ranks' stats records and ONE launch that folds them
        and fake-quantizes (distributed.observe_gather_fake_quant); None when it does not
        apply (then collect_qparameter + quantize below)."""
        from ..distributed import ObserveGatherFakeQuantFn, observe_gather_fake_quant
        from .uniform import UniformQuantizer
        obs = self.observer
        if not (self.dist_group is not None and not self.dist_defer and self.is_quantize
                and not self.is_learning_scale and self.is_observer_qparam
                and type(self.quantizer) is UniformQuantizer and isinstance(obs, MinMaxObserver)
                and not isinstance(obs, PerChannelMinMaxObserver) and self._device_observer(x)
                and x.dtype == torch.float32 and x.numel() > 0):
            return None
        self._join()
        self._x_device = x.device
        if obs._obs_stream is not None and obs._obs_stream != torch.cuda.current_stream(x.device):
            obs._join()
        state = obs.device_state(x.device)
        q = self.quantizer
        if x.requires_grad and torch.is_grad_enabled():
            y, qp, st = ObserveGatherFakeQuantFn.apply(x, state, obs.symmetric, obs.num_bits, obs.eps, q.qmin,
                                                       q.qmax, act, self.dist_group)
        else:
            y, qp, st, _ = observe_gather_fake_quant(x, state, symmetric=obs.symmetric, num_bits=obs.num_bits,
                                                     eps=obs.eps, qmin=q.qmin, qmax=q.qmax, act=act,
                                                     group=self.dist_group)
        obs._dirty = True
        self._record_stats(st[H.ST_MEANABS:H.ST_STD + 1])
        self.scale, self.zero_point = qp[H.QP_SCALE], qp[H.QP_ZP]
        return y

    def _observe_quantize_small(self, x, act):
        """Observe + quantize of a small tensor in one call (K8 / K9) when this call is the
        reference's per-call observe+quantize (qm.py:73-90) with this package's per-tensor
        MinMaxObserver and UniformQuantizer, single GPU; None when it does not apply."""
        from ..fakequant import ObserveFakeQuantFn, observe_fake_quant, observe_fq_parts_max_elems
        from .uniform import UniformQuantizer
        obs = self.observer
        if not (self.is_quantize and not self.is_learning_scale and self.is_observer_qparam
                and type(self.quantizer) is UniformQuantizer and isinstance(obs, MinMaxObserver)
                and not isinstance(obs, PerChannelMinMaxObserver) and self._device_observer(x)
                and self.dist_group is None and not self.dist_defer and x.dtype == torch.float32
                and 0 < x.numel() <= min(_OBSERVE_FQ_MAX, observe_fq_parts_max_elems())):
            return None
        self._join()
        self._x_device = x.device
        if obs._obs_stream is not None and obs._obs_stream != torch.cuda.current_stream(x.device):
            obs._join()
        state = obs.device_state(x.device)
        q = self.quantizer
        if x.requires_grad and torch.is_grad_enabled():
            y, qp, st = ObserveFakeQuantFn.apply(x, obs.symmetric, obs.num_bits, obs.eps, q.qmin, q.qmax, state,
                                                 act)
        else:
            y, qp, st, _, _ = observe_fake_quant(x, symmetric=obs.symmetric, num_bits=obs.num_bits, eps=obs.eps,
                                                 qmin=q.qmin, qmax=q.qmax, run_minmax=state, act=act)
        obs._dirty = True
        self._record_stats(st[H.ST_MEANABS:H.ST_STD + 1], x, act)
        self.scale, self.zero_point = qp[H.QP_SCALE], qp[H.QP_ZP]
        return y

    # ------------------------------------------------------------------ learnable qparams
    def _home_device(self):
        """Device of the tensors this manager observed (or of its observer state), if any."""
        dev = self.__dict__.get("_x_device")
        if dev is not None:
            return dev
        st = getattr(self.observer, "_state", None)
        if isinstance(st, torch.Tensor):
            return st.device
        for t in (self.scale, self.zero_point):
            if isinstance(t, torch.Tensor):
                return t.device
        return None

    def make_learn_qparameter(self):
        """scale -> nn.Parameter (qm.py:92-103); float64 when it came from the learn init.

        The reference creates it on the CPU and relies on a later ``model.to(device)``; here
        it is created where the observer state lives, so a model that is not moved again
        does not read its scale back to the host on every call (and stays graph-capturable)."""
        self._join()
        dev = self._home_device()
        s = self.scale
        s = s.detach().clone() if isinstance(s, torch.Tensor) else torch.tensor(s)
        self.scale = nn.Parameter(s.to(dev) if dev is not None else s, requires_grad=True)
        learn_zp = (not self.is_symmetric) or getattr(self.quantizer, "learns_zero_point", False)
        if learn_zp:
            z = self.zero_point
            z = (z.detach().to(torch.float64).clone() if isinstance(z, torch.Tensor)
                 else torch.tensor(float(z), dtype=torch.float64))
            if dev is not None:
                z = z.to(dev)
            self.zero_point = nn.Parameter(z + 1e-9, requires_grad=True)
        elif (isinstance(self.quantizer, PerChannelUniformQuantizer) and not self.quantizer.symmetric
              and isinstance(self.zero_point, torch.Tensor) and self.zero_point.dim() == 1):
            # asymmetric per-channel (build-defined, no reference counterpart): the
            # reference's hard-coded is_symmetric (qm.py:50) would reset zp to 0 and clamp
            # every negative weight at qmin = 0; keep the observer's per-channel zero
            # points as fixed [C] f64 tensors instead (learn them with learns_zero_point)
            z = self.zero_point.detach().to(torch.float64).clone()
            self.zero_point = z.to(dev) if dev is not None else z
        else:
            self.zero_point = 0

    def init_scaling_factor_for_learning(self):
        """scale = 2 * mean(mean_abs_x) / sqrt(2^(b-1) - 1)  (qm.py:105-112)."""
        self.scale = 2 * np.mean(self.mean_abs_x) / np.sqrt(2 ** (self.bits_width - 1) - 1)

    def winsorized_mean(self, x, lower=5, upper=95, sample_size=1000000):
        """Trimmed mean of x between two percentiles (qm.py:116-145; unused by the reference)."""
        flat = x.flatten()
        sample = flat[torch.randperm(flat.numel(), device=flat.device)[:sample_size]] \
            if flat.numel() > sample_size else flat
        lo = torch.quantile(sample, lower / 100)
        hi = torch.quantile(sample, upper / 100)
        return flat[(flat >= lo) & (flat <= hi)].mean()

    def extra_repr(self):
        return (f"quantizer={self.quantizer!r}, observer={self.observer!r}, bits={self.bits_width}, "
                f"observe={self.is_observer_qparam}, learn={self.is_learning_scale}, "
                f"quantize={self.is_quantize}")
