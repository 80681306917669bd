"""One C5 calibration batch through the reference's own entry point,
calibrate_qat_model (utils/quantize_manager.py:4-31 -> yolov8_qat.py:42-52 data_calib ->
modules/fused.py:124-134 -> quantizers/fake_quantize.py:49-50), on a 27-layer fused-ReLU
stack with the YOLOv8n backbone's activation shapes (bench.yolov8n_backbone) -- the
path the bench's C5 leg times: per layer ONE K2o launch (y = relu(c) written + the
deferred observer's records), then one deferred sync.  Synthetic conv outputs stand in
for the conv (MIOpen, out of scope): every layer's pre-activation is a fixed seeded
tensor.  Against the oracle (observers/minmax.py:32-74 restated, quantization_manager.py
:66-68 statistics): running min / max and the f64 qparams exact, mean|x| / mean / std to
1e-6, and every layer's output bit for bit relu(c) (torch's CPU relu keeps -0.0)."""
import numpy as np
import pytest
import torch
import torch.nn as nn

import bench
import vsiquantization_amd as V
from vsiquantization_amd.modules.fused import ConvBnReLU
from vsiquantization_amd.utils.quantize_manager import calibrate_qat_model, data_calib
from oracle import fakequant_np as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


class _SynthConvReLU(ConvBnReLU):
    """A fused ConvBnReLU whose conv output is a fixed tensor (the C5 stand-in)."""

    def _pre_act(self, x, weights, bias):
        self.seen_weights = weights   # the weight quantizer still ran (observe only)
        return self.synth


def _stack(batch):
    layers = []
    gen = torch.Generator(device=DEV).manual_seed(2024)
    for i, (cin, co, k, _s, h) in enumerate(bench.yolov8n_backbone()):
        m = _SynthConvReLU(nn.Conv2d(cin, co, k, bias=False), nn.BatchNorm2d(co), nn.ReLU(), "MinMaxObserver",
                           "UniformQuantizer", "MinMaxObserver", "UniformQuantizer", True, True, True, 2, 4)
        m.synth = torch.randn(batch, co, h, h, device=DEV, generator=gen) * (0.5 + 0.1 * i)
        if i == 5:
            m.synth[0, 0, 0, :4] = torch.tensor([-0.0, 0.0, 1e-40, -1e-40], device=DEV)
        layers.append(m)
    return nn.Sequential(*layers).to(DEV)


def test_c5_batch_through_calibrate_qat_model_equals_oracle():
    batch = 2
    model = _stack(batch)
    assert len(model) == 27
    outs = []
    hooks = [m.register_forward_hook(lambda mod, a, y: outs.append(y)) for m in model]
    loader = [(torch.randint(0, 256, (batch, 3, 320, 320), dtype=torch.uint8), None)]
    calibrate_qat_model(model, loader, data_calib, DEV)   # default: deferred (K2o + one sync)
    for h in hooks:
        h.remove()
    torch.cuda.synchronize()
    assert len(outs) == 27
    for i, (m, y) in enumerate(zip(model, outs)):
        c = m.synth.cpu().numpy()
        relu = np.where(c < 0, np.float32(0), c)   # F.relu on CPU: -0.0 stays -0.0
        assert np.array_equal(y.cpu().numpy().view(np.uint32), relu.view(np.uint32)), f"layer {i} y"
        qm = m.activation_quantizer
        obs = qm.observer
        mn, mx = O.observe_minmax(relu)
        assert (obs.min_val, obs.max_val) == (mn, mx), i
        s, z = O.minmax_qparams(mn, mx, True, 8)   # observer 8-bit through the manager (qm.py:42)
        assert (float(qm.scale), int(qm.zero_point)) == (s, z), i
        r64 = relu.astype(np.float64)
        np.testing.assert_allclose(qm.mean_abs_x, [np.abs(r64).mean()], rtol=1e-6)
        np.testing.assert_allclose(qm.mean_x, [r64.mean()], rtol=1e-6)
        np.testing.assert_allclose(qm.std, [r64.std(ddof=1)], rtol=1e-6)


def test_c5_calibration_default_equals_per_call_path():
    """The default (deferred K2o + sync) and the per-call observer path (K2 per call,
    defer_observers=False) give identical running state and qparams over 2 batches."""
    batch = 1
    a, b = _stack(batch), _stack(batch)
    loader = [(torch.randint(0, 256, (batch, 3, 320, 320), dtype=torch.uint8), None) for _ in range(2)]
    calibrate_qat_model(a, loader, data_calib, DEV)
    calibrate_qat_model(b, loader, data_calib, DEV, defer_observers=False)
    for ma, mb in zip(a, b):
        qa, qb = ma.activation_quantizer, mb.activation_quantizer
        assert (qa.observer.min_val, qa.observer.max_val) == (qb.observer.min_val, qb.observer.max_val)
        assert float(qa.scale) == float(qb.scale) and int(qa.zero_point) == int(qb.zero_point)
        np.testing.assert_allclose(qa.mean_abs_x, qb.mean_abs_x, rtol=1e-9)
