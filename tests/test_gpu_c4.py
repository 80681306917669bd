"""C4 at its workload: the YOLOv8n backbone's 27 ConvBnReLU quantizer pairs
(nets/yolov8.py:76-114, yolo_v8_n :224-227; modules/fused.py:112-134 +
quantizers/fake_quantize.py:62-66) through the public API against the oracle.

* activation path = F.relu then the learnable activation fake quant (uniform.py:47-56)
  as ONE fused call, UniformQuantizer(bits_a, True).quantize(c, scale, 0, True,
  act="relu") (K5 forward, K4-relu backward): the four largest layers at the full
  batch of 256 (104.9M / 52.4M / 52.4M / 52.4M elements), all 27 layers at batch 8;
* weight path = the 27 learnable weight fake quants as one multi-tensor launch each
  way (lsq_fake_quant_multi, the path of enable_multi_tensor_weights), at the 27
  weight shapes, w2 and w8.

Bars: y and grad bit-exact; the scale gradient within 1e-9 of the oracle's float64
sums of the reference's fp32 autograd terms.
"""
import numpy as np
import pytest
import torch

import bench
import vsiquantization_amd as V
from vsiquantization_amd.fakequant import LsqSpec, lsq_fake_quant_multi
from oracle import fakequant_np as O
from tests import goldens as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
LAYERS = bench.yolov8n_backbone()
BIG4 = sorted(range(len(LAYERS)), key=lambda i: -LAYERS[i][1] * LAYERS[i][4] ** 2)[:4]


def _act_case(layer, batch, bits, seed):
    _, cout, _, _, h = LAYERS[layer]
    gen = torch.Generator(device=DEV).manual_seed(seed)
    c = torch.randn(batch, cout, h, h, device=DEV, generator=gen)
    g = torch.randn(batch, cout, h, h, device=DEV, generator=gen)
    q = V.UniformQuantizer(bits, True)
    s0 = 2 * 0.8 / (q.qmax ** 0.5)     # the manager's learn init for mean|relu(c)| ~ 0.4
    s = torch.nn.Parameter(torch.tensor(s0, dtype=torch.float64, device=DEV))
    x = c.clone().requires_grad_(True)
    y = q.quantize(x, s, 0, True, act="relu")
    y.backward(g)
    torch.cuda.synchronize()
    # oracle: relu, learnable fq fwd/bwd, relu backward (fused.py:133, uniform.py:47-56)
    cn, gn = c.cpu().numpy(), g.cpu().numpy()
    a = O.act_forward(cn, "relu")
    gs = O.grad_scale(q.qmax, a.size)
    yo, gao, gso, _ = O.lsq_forward_backward(a, gn, s0, 0, q.qmin, q.qmax, gs)
    del a
    gco = O.act_backward(gao, cn, "relu")
    G.assert_bitwise_f32(y.detach().cpu().numpy(), yo, "y")
    G.assert_bitwise_f32(x.grad.cpu().numpy(), gco, "grad_c")
    assert abs(float(s.grad) - gso) <= 1e-9 * abs(gso), (float(s.grad), gso)


@pytest.mark.parametrize("layer", BIG4)
def test_c4_full_batch_largest_layers(layer):
    _act_case(layer, 256, 4, 100 + layer)


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("layer", range(len(LAYERS)))
def test_c4_all_layers_batch8(layer, bits):
    _act_case(layer, 8, bits, 300 + layer)


@pytest.mark.parametrize("bits_w", [2, 8])
def test_c4_multi_tensor_weights(bits_w):
    gen = torch.Generator(device=DEV).manual_seed(7 + bits_w)
    ws, gws, specs, params = [], [], [], []
    qmax = 2 ** (bits_w - 1) - 1
    for cin, cout, k, _, _ in LAYERS:
        w = torch.randn(cout, cin, k, k, device=DEV, generator=gen) * (2.0 / (cin * k * k)) ** 0.5
        s0 = float(w.abs().mean()) * 2 / qmax ** 0.5            # qm.py:112 init
        p = torch.nn.Parameter(torch.tensor(s0, dtype=torch.float64, device=DEV))
        ws.append(w.requires_grad_(True))
        gws.append(torch.randn(w.shape, device=DEV, generator=gen))
        params.append((p, s0))
        specs.append(LsqSpec(p, 0, -qmax - 1, qmax, (qmax * w.numel()) ** -0.5, False))
    ys = lsq_fake_quant_multi(ws, specs)
    torch.autograd.backward(list(ys), gws)
    torch.cuda.synchronize()
    for w, gw, y, (p, s0), sp in zip(ws, gws, ys, params, specs):
        yo, gxo, gso, _ = O.lsq_forward_backward(w.detach().cpu().numpy(), gw.cpu().numpy(), s0, 0,
                                                 sp.qmin, sp.qmax, sp.gscale)
        G.assert_bitwise_f32(y.detach().cpu().numpy(), yo, f"y {tuple(w.shape)}")
        G.assert_bitwise_f32(w.grad.cpu().numpy(), gxo, f"grad_w {tuple(w.shape)}")
        assert abs(float(p.grad) - gso) <= 1e-9 * abs(gso), (tuple(w.shape), float(p.grad), gso)


def test_c4_backbone_shapes():
    assert len(LAYERS) == 27
    sizes = sorted((LAYERS[i][1] * LAYERS[i][4] ** 2 * 256 for i in BIG4), reverse=True)
    assert sizes == [104_857_600, 52_428_800, 52_428_800, 52_428_800]
    assert np.isclose(sum(co * h * h for _, co, _, _, h in LAYERS), 2_137_600)
