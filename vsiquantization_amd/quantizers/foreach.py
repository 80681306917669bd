"""Multi-tensor weight fake quant for a whole model (MI355X extension, no reference
counterpart; the arithmetic is the reference's, quantizers/uniform.py:47-56).

In the reference every fused layer fake-quantizes its own weight on every forward
(quantizers/fake_quantize.py:62-63 -> QuantizationManager.quantize, qm.py:73-90),
and autograd runs one backward per weight.  A YOLOv8n weight is 432-295k elements:
each such launch is pure fixed cost on MI355X (4.6 us forward, 6-7 us backward).
Weights do not depend on the activations, so all of them can be fake-quantized up
front in ONE launch, and since nothing reads a weight's gradient before the
optimizer step, all their backwards can run in ONE launch when autograd reaches the
multi-output node (k_multi.hip).  Per tensor the results are bit-identical to the
per-layer path.

    handle = enable_multi_tensor_weights(model)   # forward pre-hook on the model
    ...train...
    handle.remove()

Only layers whose weight quantizer is in the learnable per-tensor mode
(``is_learning_scale``; UniformQuantizer / LSQQuantizer) are batched; every other
layer keeps its own path.
"""
from __future__ import annotations

import weakref

import torch

from ..fakequant import LsqSpec, lsq_fake_quant_multi
from .fake_quantize import FakeQuantize
from .per_channel import PerChannelUniformQuantizer
from .quantization_manager import QuantizationManager
from .uniform import UniformQuantizer


def _weight_spec(layer):
    """(weight, LsqSpec) when the layer's weight fake quant can join a multi-tensor
    launch, else None (quantizer off -- is_quantize False returns the weight unquantized,
    qm.py:86-90 -- or not learnable / per-tensor / on the GPU)."""
    qm = getattr(layer, "weight_quantizer", None)
    if not isinstance(qm, QuantizationManager) or not qm.is_learning_scale or not qm.is_quantize:
        return None
    q = qm.quantizer
    if not isinstance(q, UniformQuantizer) or isinstance(q, PerChannelUniformQuantizer):
        return None
    w, _ = layer.get_weight_bias()
    if not (isinstance(w, torch.Tensor) and w.is_cuda and w.dtype == torch.float32 and w.numel() > 0):
        return None
    s = qm.scale
    if isinstance(s, torch.Tensor) and (s.numel() != 1 or s.device != w.device):
        return None
    qm._join()
    gscale, zp, learn_zp = q.learn_args(w, qm.zero_point)
    if learn_zp == 2:   # a zero point used as given with its gradient: the per-layer path (K4 mode 2)
        return None
    return w, LsqSpec(s, zp, q.qmin, q.qmax, gscale, learn_zp)


def quantize_weights_multi(layers) -> int:
    """Fake-quantize the weights of every eligible layer in one launch and hand each
    layer its result for its next forward (FakeQuantize.quantize_weights).  Returns the
    number of layers batched."""
    picked = []
    for m in layers:
        r = _weight_spec(m)
        if r is not None:
            picked.append((m, *r))
    if not picked:
        return 0
    ys = lsq_fake_quant_multi([w for _, w, _ in picked], [sp for _, _, sp in picked])
    for (m, w, _), y in zip(picked, ys):
        m._weight_stash = (w, y)
    return len(picked)


class NoHandle:
    """Returned by an enable_* call on a model that already has that hook."""

    def remove(self):
        pass


class ModelHook:
    """Base of the model-level launch hooks (K7 here, K4d in deferred.py): a callable
    object rather than a closure, so a model carrying it still pickles (whole-model
    torch.save) and a deep copy (EMA / teacher) gets a fresh hook with its own cache.
    ``vsiq_model_launch`` marks it for utils.quantize_manager.disable_model_launches.
    Module lists are cached per hooked module (weakly): walking the module tree on every
    forward cost ~0.1 ms of host time per step."""

    vsiq_model_launch = True

    def __init__(self, model=None):
        self._cache = weakref.WeakKeyDictionary()
        if model is not None:
            self._cache[model] = self.collect(model)

    def collect(self, mod):
        raise NotImplementedError

    def items(self, mod):
        ms = self._cache.get(mod)
        if ms is None:
            ms = self._cache[mod] = self.collect(mod)
        return ms

    def __getstate__(self):
        return {}

    def __setstate__(self, state):
        self._cache = weakref.WeakKeyDictionary()

    def __deepcopy__(self, memo):
        return type(self)()


class MultiWeightsHook(ModelHook):
    """Forward pre-hook: quantize_weights_multi over the model's FakeQuantize layers."""

    def collect(self, mod):
        return [m for m in mod.modules() if isinstance(m, FakeQuantize)]

    def __call__(self, mod, args):
        quantize_weights_multi(self.items(mod))


def enable_multi_tensor_weights(model):
    """Register a forward pre-hook on ``model`` that runs quantize_weights_multi over its
    FakeQuantize layers before every forward.  Returns the hook handle.  The layer list is
    taken now; a layer added later quantizes its weight per call, which gives the same
    values, so enable again after changing the model's structure only to batch it too.  A
    deep copy of the model batches its own layers.  Already enabled: nothing is added
    (the returned handle removes nothing)."""
    if any(isinstance(h, MultiWeightsHook) for h in model._forward_pre_hooks.values()):
        return NoHandle()
    return model.register_forward_pre_hook(MultiWeightsHook(model))
