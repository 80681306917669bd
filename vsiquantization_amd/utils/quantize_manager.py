"""QAT lifecycle switches (reference: utils/quantize_manager.py:4-117).

Layers are found by duck typing (``hasattr(module, "weight_quantizer")`` /
``"activation_quantizer"``) exactly like the reference, and the three manager
flags select the kernel branch:

  calibrate_qat_model       observe only        (K2 / K3 observe, no fake quant)
  activate_learning_qparam  learn-init + Parameters  (K1 fwd + K4 bwd from then on)
  activate_quantizer        fake quant on
"""


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


def activate_learning_qparam(model, layer_names=None, use_init=True, active=True):
    """Set ``is_learning_scale``; optionally re-init scale from mean|x|; make Parameters."""
    for name, module in model.named_modules():
        if layer_names is not None and name not in layer_names:
            continue
        for qm in _managers(module):
            qm.is_learning_scale = active
            if use_init:
                qm.init_scaling_factor_for_learning()
            if active:
                qm.make_learn_qparameter()


def deactivate_learning_qparam(model, layer_names=None):
    activate_learning_qparam(model, layer_names=layer_names, active=False)


def activate_quantizer(model, layer_names=None, active=True):
    for name, module in model.named_modules():
        if layer_names is not None and name not in layer_names:
            continue
        for qm in _managers(module):
            qm.is_quantize = active


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
