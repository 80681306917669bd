"""QAT lifecycle switches (reference: utils/quantize_manager.py:4-117).

Layers are found by duck typing (``hasattr(module, "weight_quantizer")`` /
``"activation_quantizer"``) exactly like the reference, and the three manager
flags select the kernel branch:

  calibrate_qat_model       observe only        (K2 / K3 observe, no fake quant)
  activate_learning_qparam  learn-init + Parameters  (K1 fwd + K4 bwd from then on)
  activate_quantizer        fake quant on

Entering training (activate_learning_qparam / activate_quantizer, the reference's
sequence before its training loop, yolov8_qat.py:90-92) also turns on the model-level
launches, with no call in user code: every learnable weight quantizer of the model in
ONE forward and ONE backward launch (K7, quantizers/foreach.py) and every learnable
quantizer's scale / zero-point gradient folded in ONE launch per backward (K4d,
quantizers/deferred.py).  Outputs and input gradients are bit-identical to the per-call
path, qparam gradients equal to float64 summation order.  Opt out per call
(``model_launches=False``), per process (VSIQ_MODEL_LAUNCHES=0) or per model
(``disable_model_launches``).
"""
import os


def _managers(module):
    for attr in ("weight_quantizer", "activation_quantizer"):
        if hasattr(module, attr):
            yield getattr(module, attr)


def join_observers(model):
    """Make the current stream wait for every manager's queued (side-stream) observer work."""
    for module in model.modules():
        for qm in _managers(module):
            if hasattr(qm, "_join"):
                qm._join()


def calibrate_qat_model(model, dataloader, data_calib, device=None, async_observers=False,
                        defer_observers=True):
    """Observe-only mode on every manager, eval(), then ``data_calib(model, dataloader, device)``.

    MI355X options (results identical either way; ``defer_observers`` is on by default
    since nothing reads an observer before calibration ends -- utils/quantize_manager.py
    :4-31 in the reference -- and the deferred pass is ~2x cheaper per call):
    * ``async_observers``: queue each observer pass on a side stream
      (``QuantizationManager.async_observer``) so the next layers do not wait for its
      reduction tail; all are joined before returning.  Costs ~10 us of host time per
      call (stream hand-off), which only pays when the model's own kernels are short
      enough that the observers' tails are exposed.
    * ``defer_observers``: per-tensor observers write partial records only (K2p: no
      cross-workgroup fold, no atomics, no running update per call) and ONE
      ``distributed.sync_calibration`` at the end folds every call of every layer,
      all-reduces across ranks where a manager has a ``dist_group``, and replays the
      running min/max exactly (minmax.py:42-47)."""
    mgrs = []
    for module in model.modules():
        for qm in _managers(module):
            qm.is_observer_qparam = True
            qm.is_learning_scale = False
            qm.is_quantize = False
            if hasattr(qm, "async_observer"):
                mgrs.append((qm, qm.async_observer, qm.dist_defer))
                qm.async_observer = async_observers
                qm.dist_defer = qm.dist_defer or defer_observers
    model.eval()
    try:
        data_calib(model, dataloader, device)
    finally:
        for qm, prev, prev_defer in mgrs:
            qm.async_observer = prev
            qm.dist_defer = prev_defer
        join_observers(model)
    if defer_observers:
        from ..distributed import sync_calibration
        sync_calibration(model)


def enable_model_launches(model):
    """Install the model-level launches on ``model`` (forward hooks; idempotent): K7 for
    the learnable weight quantizers and K4d for the learnable qparam gradients.  Which
    managers join is decided per forward (learnable, quantizing, per-tensor, on the GPU);
    every other manager keeps its per-call path."""
    from ..quantizers.deferred import enable_deferred_qparam_grads
    from ..quantizers.foreach import enable_multi_tensor_weights
    enable_multi_tensor_weights(model)
    enable_deferred_qparam_grads(model)


def disable_model_launches(model):
    """Remove the model-level launch hooks (K7 / K4d) from ``model``: every manager takes
    its per-call path again (same outputs; qparam gradients to float64 summation order)."""
    from ..quantizers.deferred import _managers as _all_managers
    from ..quantizers.deferred import clear_bundled
    for hooks in (model._forward_pre_hooks, model._forward_hooks):
        for k in [k for k, h in hooks.items() if getattr(h, "vsiq_model_launch", False)]:
            del hooks[k]
    clear_bundled(_all_managers(model))


def model_launches_enabled(model) -> bool:
    return any(getattr(h, "vsiq_model_launch", False) for h in model._forward_pre_hooks.values())


def _auto_model_launches(model, model_launches):
    if model_launches is None:
        model_launches = os.environ.get("VSIQ_MODEL_LAUNCHES", "1") != "0"
    if model_launches:
        enable_model_launches(model)


def activate_learning_qparam(model, layer_names=None, use_init=True, active=True, model_launches=None):
    """Set ``is_learning_scale``; optionally re-init scale from mean|x|; make Parameters.
    Activating also installs the model-level launches (module docstring; ``model_launches``
    False or VSIQ_MODEL_LAUNCHES=0: not)."""
    for name, module in model.named_modules():
        if layer_names is not None and name not in layer_names:
            continue
        for qm in _managers(module):
            qm.is_learning_scale = active
            if use_init:
                qm.init_scaling_factor_for_learning()
            if active:
                qm.make_learn_qparameter()
    if active:
        _auto_model_launches(model, model_launches)


def deactivate_learning_qparam(model, layer_names=None):
    activate_learning_qparam(model, layer_names=layer_names, active=False)


def activate_quantizer(model, layer_names=None, active=True, model_launches=None):
    """Set ``is_quantize``; activating also installs the model-level launches (see
    activate_learning_qparam)."""
    for name, module in model.named_modules():
        if layer_names is not None and name not in layer_names:
            continue
        for qm in _managers(module):
            qm.is_quantize = active
    if active:
        _auto_model_launches(model, model_launches)


def deactivate_quantizer(model, layer_names=None):
    activate_quantizer(model, layer_names=layer_names, active=False)


def data_calib(model, calib_loader, device, num_batches=16):
    """Restatement of yolov8_qat.py:42-52: eval, <=16 batches of uint8 images / 255, train().

    ``calib_loader`` yields ``(imgs, targets)`` with uint8 NCHW images."""
    model.eval()
    model.to(device)
    for i, (imgs, _targets) in enumerate(calib_loader):
        model(imgs.to(device, non_blocking=True).float() / 255.0)
        if i == num_batches - 1:
            break
    model.train()


def load_partial_checkpoint(model, checkpoint_path):
    """Load the entries of a saved state_dict whose names and shapes match the model
    (reference: utils/util.py:17-40).  The learnable qparams are float64 Parameters named
    ``<layer>.weight_quantizer.scale`` / ``.activation_quantizer.scale`` once
    activate_learning_qparam has run (yolov8_qat.py:299 saves them).  Loads with
    ``weights_only=True`` (tensors only, nothing executed from the file)."""
    import torch
    checkpoint_state_dict = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    model_state_dict = model.state_dict()
    matched = {}
    for name, param in checkpoint_state_dict.items():
        if name in model_state_dict:
            if model_state_dict[name].shape == param.shape:
                matched[name] = param
            else:
                print(f"Skip loading parameter: {name} due to shape mismatch "
                      f"({param.shape} vs {model_state_dict[name].shape})")
        else:
            print(f"Skip loading parameter: {name} as it's not in the model")
    model_state_dict.update(matched)
    model.load_state_dict(model_state_dict)
    print(f"Loaded {len(matched)} layers from checkpoint.")
    return len(matched)
