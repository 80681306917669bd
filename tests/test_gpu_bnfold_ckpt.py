"""BN fold on the device (bit-identical to the torch CPU fold) and the QAT state_dict
round trip (learnable f64 scale Parameters, load_partial_checkpoint)."""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

from vsiquantization_amd.modules.fused import ConvBnReLU, LinearBnReLU, _bn_fold
from vsiquantization_amd.utils.quantize_manager import (activate_learning_qparam, activate_quantizer,
                                                        calibrate_qat_model, data_calib,
                                                        load_partial_checkpoint)

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _bn(c, seed):
    torch.manual_seed(seed)
    bn = nn.BatchNorm2d(c, eps=1e-3)
    bn.running_mean.uniform_(-0.3, 0.3)
    bn.running_var.uniform_(0.2, 3.0)
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.uniform_(-0.2, 0.2)
    return bn


def _fold_ieee(w, b, bn):
    """The reference fold (fused.py:100-108) as IEEE fp32 numpy ops, step by step."""
    f32 = np.float32
    std = np.sqrt((bn.running_var.numpy() + f32(bn.eps)).astype(f32)).astype(f32)
    f = (bn.weight.detach().numpy() / std).astype(f32)
    wf = (w.numpy() * f.reshape([-1] + [1] * (w.dim() - 1))).astype(f32)
    bb = b.numpy() if isinstance(b, torch.Tensor) else f32(0)
    bf = (bn.bias.detach().numpy() + ((bb - bn.running_mean.numpy()).astype(f32) * f).astype(f32)).astype(f32)
    return wf, bf


@pytest.mark.parametrize("shape,bias", [((64, 32, 3, 3), False), ((16, 3, 3, 3), True), ((256, 512), True),
                                        ((7, 5, 1, 1), False)])
def test_bn_fold_device_bitwise(shape, bias):
    """Bit-identical to IEEE fp32 in the reference's order.  (torch's own CPU fold is
    not IEEE on every host -- on the MI355X box's AVX-512 CPU it differs in the last
    bit for some channels -- so the IEEE restatement is the checker.)"""
    torch.manual_seed(1)
    w = torch.randn(shape)
    b = torch.randn(shape[0]) if bias else 0
    bn = _bn(shape[0], 2)
    view = [-1] + [1] * (len(shape) - 1)
    wd, bd = _bn_fold(w.to(DEV), b.to(DEV) if bias else 0, copy.deepcopy(bn).to(DEV), view)
    wi, bi = _fold_ieee(w, b, bn)
    assert np.array_equal(wd.cpu().numpy().view(np.uint32), wi.view(np.uint32))
    assert np.array_equal(bd.cpu().numpy().view(np.uint32), bi.view(np.uint32))


def _model():
    torch.manual_seed(0)
    layers = []
    for cin, cout in ((3, 8), (8, 16)):
        cv = nn.Conv2d(cin, cout, 3, padding=1, bias=False)
        layers.append(ConvBnReLU(cv, _bn(cout, cout), nn.ReLU(), "MinMaxObserver", "UniformQuantizer",
                                 "MinMaxObserver", "UniformQuantizer", True, True, True, 4, 4))
    return nn.Sequential(*layers).to(DEV)


def _loader():
    g = torch.Generator().manual_seed(5)
    return [(torch.randint(0, 256, (2, 3, 16, 16), generator=g, dtype=torch.uint8), None) for _ in range(3)]


def test_state_dict_round_trip(tmp_path):
    a = _model()
    calibrate_qat_model(a, _loader(), data_calib, DEV)
    activate_learning_qparam(a)
    activate_quantizer(a)
    sd = a.state_dict()
    assert sd["0.weight_quantizer.scale"].dtype == torch.float64
    assert sd["1.activation_quantizer.scale"].dtype == torch.float64
    x = torch.rand(2, 3, 16, 16, device=DEV)
    opt = torch.optim.SGD(a.parameters(), lr=1e-3)
    a(x).square().mean().backward()
    opt.step()
    path = tmp_path / "last_qat.pth"
    torch.save(a.state_dict(), path)
    b = _model()
    calibrate_qat_model(b, _loader(), data_calib, DEV)
    activate_learning_qparam(b)
    activate_quantizer(b)
    n = load_partial_checkpoint(b, str(path))
    assert n == len(a.state_dict())
    a.eval(), b.eval()
    with torch.no_grad():
        assert torch.equal(a(x), b(x))


def test_linear_bn_fold_on_device():
    torch.manual_seed(3)
    lin = nn.Linear(40, 24)
    bn = nn.BatchNorm1d(24)
    bn.running_var.uniform_(0.5, 2.0)
    h = LinearBnReLU(copy.deepcopy(lin), copy.deepcopy(bn), nn.ReLU(), "MinMaxObserver", "UniformQuantizer",
                     "MinMaxObserver", "UniformQuantizer")
    d = LinearBnReLU(copy.deepcopy(lin).to(DEV), copy.deepcopy(bn).to(DEV), nn.ReLU(), "MinMaxObserver",
                     "UniformQuantizer", "MinMaxObserver", "UniformQuantizer")
    wi, bi = _fold_ieee(lin.weight.detach(), lin.bias.detach(), bn)
    assert np.array_equal(d.linear_fuse.weight.detach().cpu().numpy().view(np.uint32), wi.view(np.uint32))
    assert np.array_equal(d.linear_fuse.bias.detach().cpu().numpy().view(np.uint32), bi.view(np.uint32))
    torch.testing.assert_close(d.linear_fuse.weight.detach().cpu(), h.linear_fuse.weight.detach())
