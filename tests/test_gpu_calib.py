"""Calibration on MI355X: side-stream (async) observers give exactly the synchronous
results; the fused-ReLU observer path through calibrate_qat_model."""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

from vsiquantization_amd.modules.fused import ConvBnReLU
from vsiquantization_amd.utils.quantize_manager import calibrate_qat_model, data_calib

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _model():
    torch.manual_seed(0)
    layers = []
    for cin, cout in ((3, 16), (16, 32), (32, 32)):
        cv = nn.Conv2d(cin, cout, 3, padding=1, bias=False)
        bn = nn.BatchNorm2d(cout)
        bn.running_var.uniform_(0.5, 2.0)
        layers.append(ConvBnReLU(cv, bn, nn.ReLU(), "MinMaxObserver", "UniformQuantizer", "MinMaxObserver",
                                 "UniformQuantizer", True, True, True, 4, 4))
    return nn.Sequential(*layers).to(DEV)


def _loader(n=6):
    g = torch.Generator().manual_seed(1)
    return [(torch.randint(0, 256, (4, 3, 32, 32), generator=g, dtype=torch.uint8), None) for _ in range(n)]


def _state(model):
    out = []
    for m in model:
        for qm in (m.weight_quantizer, m.activation_quantizer):
            out.append((qm.observer.min_val, qm.observer.max_val, list(qm.mean_abs_x), list(qm.mean_x),
                        list(qm.std)))
    return out


def test_async_observers_equal_sync():
    a = _model()
    b = copy.deepcopy(a)
    calibrate_qat_model(a, _loader(), data_calib, DEV, async_observers=True)
    calibrate_qat_model(b, _loader(), data_calib, DEV, async_observers=False)
    sa, sb = _state(a), _state(b)
    assert sa == sb
    assert all(len(s[2]) == 6 for s in sa)
    # the flag is restored and nothing stays pending
    assert all(not m.activation_quantizer.async_observer for m in a)
    assert all(m.activation_quantizer._side is None for m in a)
