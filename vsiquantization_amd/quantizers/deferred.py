"""Deferred learnable-qparam gradient fold for a whole model (K4d; MI355X extension, no
reference counterpart -- the arithmetic is the reference's, quantizers/uniform.py:47-56
with ScaleGradient :242-255).

In the reference every learnable quantizer's backward produces its scale (and zero
point) gradient right away (autograd of uniform.py:47-56).  On MI355X that gradient is a
device-wide reduction: K4 ends every launch with a record drain, arrival atomics and a
last-workgroup fold, 3-5 us per launch at 2-26M elements (C4's 27 activation quantizers:
~135 us of a 1.28 ms backward).  Nothing reads those gradients before the optimizer,
so this mode runs each quantizer's backward records-only (vsiq_act_lsq_bwd_part_f32:
grad_x bit-identical, one record per workgroup, no reduction) and folds every
quantizer's records in ONE launch (vsiq_lsq_fold_multi) when autograd reaches a bundle
node that sits between the model's f64 ``scale`` / ``zero_point`` Parameters and their
uses.  The bundle's backward runs once all of its uses have delivered their (record)
gradients, then hands the folded values to autograd: AccumulateGrad, DDP's bucket hooks
and gradient accumulation see ordinary gradients.

    handle = enable_deferred_qparam_grads(model)   # forward pre-hook on the model
    ...train...
    handle.remove()

Each manager uses its bundled qparams for the FIRST learnable call of a forward; a second
call in the same forward takes the per-call path (a placeholder gradient must reach the
bundle unsummed).  Eligible managers: learnable per-tensor UniformQuantizer / LSQQuantizer
with a 0-dim float64 CUDA scale (and zero point, when learned) and a scalar gradient scale.
"""
from __future__ import annotations

import torch

from .. import _hip as H
from ..fakequant import fake_quant, scalar_source
from .foreach import ModelHook, NoHandle
from .per_channel import PerChannelUniformQuantizer
from .quantization_manager import QuantizationManager
from .uniform import UniformQuantizer

# grad_out storage pointer -> pending fold of one records-only backward.  A backward
# that never reaches the bundle (torch.autograd.grad for the activations only) leaves
# its entries behind; the oldest are dropped beyond _PENDING_MAX (a real step holds one
# per quantizer of the model).
_PENDING = {}
_PENDING_MAX = 1 << 14
# forward generation (bundle_qparams): a pending entry is consumed by the bundle within
# the backward pass that created it, so entries older than the previous generation are
# orphans of a backward that never reached the bundle and are dropped at the next forward
# (one generation of slack: a checkpointed layer re-runs its forward inside the backward)
_GEN = [0]


class _Fold:
    __slots__ = ("records", "nrec", "zd", "zh", "gscale", "qmin", "qmax", "learn_zp", "out", "keep", "gen")


def lsq_backward_part(g, x, scale, zero_point, qmin, qmax, learn_zp, act, records):
    """K4 records-only: grad_x; the call's per-workgroup {sum t, sum z} into ``records``."""
    g = H.require_device_f32(g, "grad_output")
    dev = g.device
    gx = torch.empty_like(g)
    sd, sh = scalar_source(scale, dev)
    zd, zh = scalar_source(zero_point, dev)
    rc = H.lib().vsiq_act_lsq_bwd_part_f32(H.ptr(g), H.ptr(x), H.ptr(gx), H.c_i64(g.numel()), H.act_code(act),
                                           H.ptr(sd), sh, H.ptr(zd), zh, int(bool(learn_zp)), int(qmin), int(qmax),
                                           H.ptr(records), H.c_i64(records.numel()), H.stream_of(dev))
    H.check(rc, "vsiq_act_lsq_bwd_part_f32")
    return gx, zd, zh


def fold(entries) -> None:
    """ONE launch (per 64 calls): every pending call's records -> its grad_out[2]."""
    if not entries:
        return
    arr = (H.LsqFold * len(entries))()
    for i, e in enumerate(entries):
        arr[i] = H.LsqFold(e.records.data_ptr(), e.nrec, e.zd.data_ptr() if e.zd is not None else None, e.zh,
                           e.gscale, e.out.data_ptr(), e.qmin, e.qmax, int(e.learn_zp), 0)
    rc = H.lib().vsiq_lsq_fold_multi(arr, len(entries), H.stream_of(entries[0].out.device))
    H.check(rc, "vsiq_lsq_fold_multi")


class DeferredLearnFn(torch.autograd.Function):
    """FakeQuantLearnFn with the records-only backward: the qparam gradients it returns
    are placeholders (views of a pending f64[2]) that the bundle folds.  The Python form
    of the C++ node fq_learn_deferred (VSIQ_TORCH_EXT=0; tests compare the two)."""

    @staticmethod
    def forward(ctx, x, scale, zero_point, qmin, qmax, gscale, learn_zp, act):
        x = H.require_device_f32(x)
        y, _, _ = fake_quant(x, scale, zero_point, qmin, qmax, zp_round=learn_zp, act=act)
        ctx.save_for_backward(x)
        ctx.scale, ctx.zp = scale, zero_point
        ctx.args = (qmin, qmax, gscale, learn_zp, act)
        return y

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        qmin, qmax, gscale, learn_zp, act = ctx.args
        s, z = ctx.scale, ctx.zp
        dev = x.device
        e = _Fold()
        e.nrec = int(H.lib().vsiq_lsq_part_records(H.c_i64(x.numel())))
        e.records = torch.empty(2 * e.nrec, dtype=torch.float64, device=dev)
        gx, e.zd, e.zh = lsq_backward_part(gy.contiguous(), x, s, z, qmin, qmax, learn_zp, act, e.records)
        e.gscale, e.qmin, e.qmax, e.learn_zp = float(gscale), int(qmin), int(qmax), bool(learn_zp)
        e.out = torch.empty(2, dtype=torch.float64, device=dev)
        e.keep = (s, z)
        e.gen = _GEN[0]
        _PENDING[e.out.data_ptr()] = e
        while len(_PENDING) > _PENDING_MAX:
            _PENDING.pop(next(iter(_PENDING)))
        gs = e.out[0].view(s.shape) if ctx.needs_input_grad[1] else None
        gz = e.out[1].view(z.shape) if (learn_zp and isinstance(z, torch.Tensor) and ctx.needs_input_grad[2]) else None
        return gx, gs, gz, None, None, None, None, None


def deferred_learn(x, scale, zero_point, qmin, qmax, gscale, learn_zp, act):
    """Learnable fake quant whose backward is records-only (K4d): the C++ node of
    _vsiq_torch.so (FqLearnDeferredBackward, no Python in the backward), or
    DeferredLearnFn with VSIQ_TORCH_EXT=0."""
    if H.torch_ext_enabled():
        x = H.require_device_f32(x)
        cuda_z = isinstance(zero_point, torch.Tensor) and zero_point.device.type == "cuda"
        zt = zero_point if cuda_z else None   # a CPU tensor / number: its host value (scalar_source)
        zh = 0.0 if cuda_z else float(zero_point)
        return H.torch_ext().fq_learn_deferred(x, scale, zt, zh, int(qmin), int(qmax), float(gscale),
                                               bool(learn_zp), H.act_code(act))
    return DeferredLearnFn.apply(x, scale, zero_point, qmin, qmax, gscale, learn_zp, act)


def pending_count() -> int:
    """Records-only backwards waiting for their bundle's fold (Python and C++ nodes)."""
    n = len(_PENDING)
    if H.torch_ext_enabled():
        n += int(H.torch_ext().deferred_pending())
    return n


class QParamBundleFn(torch.autograd.Function):
    """Identity on the model's learnable qparams; its backward folds every pending
    records-only backward in one launch and returns the folded gradients."""

    @staticmethod
    def forward(ctx, *params):
        ctx.set_materialize_grads(False)   # a qparam not used this forward: None, not zeros
        return tuple(p.view_as(p) for p in params)

    @staticmethod
    def backward(ctx, *grads):
        entries, seen, native = [], set(), []
        for g in grads:
            if g is None:
                continue
            p = g.data_ptr()
            e = _PENDING.get(p) or _PENDING.get(p - 8)
            if e is None:
                native.append(p)   # a C++ node's pending call (or an error, below)
            elif id(e) not in seen:
                seen.add(id(e))
                entries.append(e)
        fold(entries)
        for e in entries:
            _PENDING.pop(e.out.data_ptr(), None)
        missing = len(native)
        if native and H.torch_ext_enabled():
            missing = int(H.torch_ext().deferred_fold(native))
        if missing:
            raise RuntimeError("deferred qparam gradient: a bundled scale / zero point received a "
                               "gradient that is not a pending fold (was it used twice in one forward?)")
        return grads


def _eligible(qm) -> bool:
    if not (isinstance(qm, QuantizationManager) and qm.is_learning_scale and qm.is_quantize):
        return False
    q = qm.quantizer
    if not isinstance(q, UniformQuantizer) or isinstance(q, PerChannelUniformQuantizer):
        return False
    s = qm.scale
    if not (isinstance(s, torch.Tensor) and s.requires_grad and s.is_cuda and s.dtype == torch.float64
            and s.dim() == 0):
        return False
    z = qm.zero_point
    if isinstance(z, torch.Tensor) and z.requires_grad and not (z.is_cuda and z.dtype == torch.float64
                                                                and z.dim() == 0):
        return False
    if q.symmetric and isinstance(z, torch.Tensor) and z.requires_grad and not getattr(q, "learns_zero_point", False):
        return False   # a zero point used as given with its gradient (K4 zp_learn 2): per-call path
    cal = getattr(q, "calib_grad_scale", 1)
    return not (isinstance(cal, torch.Tensor) and cal.numel() > 1)


def bundle_qparams(managers) -> int:
    """Route the eligible managers' next learnable call through one QParamBundleFn node."""
    _GEN[0] += 1
    stale = [k for k, e in _PENDING.items() if e.gen < _GEN[0] - 1]
    for k in stale:
        del _PENDING[k]
    if H.torch_ext_enabled():
        H.torch_ext().deferred_generation()
    picked = [qm for qm in managers if _eligible(qm)]
    if not picked or not torch.is_grad_enabled():
        return 0
    params, slots = [], []
    for qm in picked:
        slots.append((qm, len(params), isinstance(qm.zero_point, torch.Tensor) and qm.zero_point.requires_grad))
        params.append(qm.scale)
        if slots[-1][2]:
            params.append(qm.zero_point)
    views = QParamBundleFn.apply(*params)
    for qm, i, has_z in slots:
        qm.__dict__["_deferred_qparams"] = (views[i], views[i + 1] if has_z else qm.zero_point)
    return len(picked)


def _managers(model):
    return [m for m in model.modules() if isinstance(m, QuantizationManager)]


def clear_bundled(managers) -> None:
    """Drop bundled qparams a forward did not use (e.g. weight quantizers served by the
    multi-tensor launch), so that no later forward picks up a finished graph's views."""
    for qm in managers:
        qm.__dict__.pop("_deferred_qparams", None)


class _Handles:
    def __init__(self, *handles):
        self.handles = handles

    def remove(self):
        for h in self.handles:
            h.remove()


class BundlePreHook(ModelHook):
    """Forward pre-hook: bundle the learnable qparams of the model's managers."""

    def collect(self, mod):
        return _managers(mod)

    def __call__(self, mod, args):
        bundle_qparams(self.items(mod))


class BundlePostHook(ModelHook):
    """Forward hook: drop the bundled qparams the forward did not use."""

    def collect(self, mod):
        return _managers(mod)

    def __call__(self, mod, args, out):
        clear_bundled(self.items(mod))


def enable_deferred_qparam_grads(model):
    """Forward hooks on ``model``: before every forward, bundle the learnable qparams of
    its QuantizationManagers (see the module docstring); after it, drop the unused ones.
    Returns a handle whose ``remove()`` removes both hooks.  The manager list is taken now;
    a manager added later takes the per-call path, which gives the same gradients, so
    enable again after changing the model's structure only to defer it too.  A deep copy
    of the model bundles its own managers.  Already enabled: nothing is added (the
    returned handle removes nothing)."""
    if any(isinstance(h, BundlePreHook) for h in model._forward_pre_hooks.values()):
        return NoHandle()
    return _Handles(model.register_forward_pre_hook(BundlePreHook(model)),
                    model.register_forward_hook(BundlePostHook(model)))
