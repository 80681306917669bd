"""The reference's own training sequence -- calibrate_qat_model, activate_learning_qparam,
activate_quantizer (yolov8_qat.py:90-92), then plain forward / backward steps
(yolov8_qat.py:225-263) -- runs the model-level launches by default: K7 (every learnable
weight quantizer in one launch each way, quantizers/foreach.py) and K4d (records-only
learnable backwards + one fold per backward, quantizers/deferred.py), with no call in user
code.  Against the same model on the per-call path (model_launches=False):

* outputs, input gradients, conv weight / bias gradients and the weight quantizers' f64
  scale gradients bit for bit (MIOpen in deterministic mode, so the upstream gradients
  are reproducible), the activation quantizers' f64 scale / zero-point gradients to
  float64 summation order (1e-12);
* the same through a deep copy (EMA / teacher), gradient accumulation over 2 micro-
  batches, GraphedStep capture + replay, and a state_dict save / load;
* the opt-outs: VSIQ_MODEL_LAUNCHES=0, model_launches=False, disable_model_launches."""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

import vsiquantization_amd as V
from vsiquantization_amd.modules.fused import ConvBnReLU
from vsiquantization_amd.quantizers import deferred as D
from vsiquantization_amd.utils.quantize_manager import (activate_learning_qparam, activate_quantizer,
                                                        calibrate_qat_model, data_calib,
                                                        load_partial_checkpoint)

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(autouse=True)
def _deterministic_convs():
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    yield
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev


def _bn(c, seed):
    torch.manual_seed(seed)
    bn = nn.BatchNorm2d(c, eps=1e-3)
    bn.running_mean.uniform_(-0.3, 0.3)
    bn.running_var.uniform_(0.2, 3.0)
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.uniform_(-0.2, 0.2)
    return bn


def _model(launches=None):
    """Three fused ConvBnReLU layers (w4/a4 sym UniformQuantizer; the last activation
    quantizer an asymmetric LSQQuantizer with a learned zero point), the reference sequence."""
    torch.manual_seed(0)
    layers = []
    for i, (cin, cout) in enumerate(((3, 16), (16, 32), (32, 32))):
        qa, asym = ("LSQQuantizer", False) if i == 2 else ("UniformQuantizer", True)
        layers.append(ConvBnReLU(nn.Conv2d(cin, cout, 3, padding=1, bias=False), _bn(cout, 10 + i), nn.ReLU(),
                                 "MinMaxObserver", "UniformQuantizer", "MinMaxObserver", qa, True, asym, True, 4, 4))
    m = nn.Sequential(*layers).to(DEV)
    gen = torch.Generator().manual_seed(1)
    loader = [(torch.randint(0, 256, (4, 3, 24, 24), generator=gen, dtype=torch.uint8), None) for _ in range(2)]
    calibrate_qat_model(m, loader, data_calib, DEV)
    activate_learning_qparam(m, use_init=True, model_launches=launches)
    activate_quantizer(m, model_launches=launches)
    m.to(DEV)
    m.train()
    return m


def _pair():
    a = _model()                  # the reference sequence: launches on by default
    b = _model(launches=False)    # the per-call path
    assert V.model_launches_enabled(a) and not V.model_launches_enabled(b)
    return a, b


def _x(seed=3, n=4):
    g = torch.Generator().manual_seed(seed)
    return (torch.randint(0, 256, (n, 3, 24, 24), generator=g, dtype=torch.uint8).float() / 255).to(DEV)


def _grads(m):
    return {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}


def _assert_same_grads(ga, gb, tag=""):
    assert ga.keys() == gb.keys(), (tag, set(ga) ^ set(gb))
    assert any(n.endswith("weight_quantizer.scale") for n in ga) and any(
        n.endswith("activation_quantizer.zero_point") for n in ga)
    for n in ga:
        if "activation_quantizer" in n:   # K4d fold vs K4's in-kernel fold: f64 summation order
            np.testing.assert_allclose(ga[n].cpu().numpy(), gb[n].cpu().numpy(), rtol=1e-12, atol=1e-300,
                                       err_msg=f"{tag} {n}")
        else:                             # K7 == per-layer K1 / K4 bit for bit
            assert torch.equal(ga[n], gb[n]), (tag, n)


def _step(m, x):
    xi = x.clone().requires_grad_(True)
    y = m(xi)
    y.square().mean().backward()
    return y.detach(), xi.grad


def test_reference_sequence_enables_model_launches_and_equals_per_call():
    a, b = _pair()
    x = _x()
    ya, gxa = _step(a, x)
    yb, gxb = _step(b, x)
    torch.cuda.synchronize()
    assert torch.equal(ya, yb) and torch.equal(gxa, gxb)
    _assert_same_grads(_grads(a), _grads(b))
    assert D.pending_count() == 0
    # a second step after an optimizer update (new weights, new scales)
    for m in (a, b):
        torch.optim.SGD(m.parameters(), lr=1e-3).step()
        m.zero_grad(set_to_none=True)
    ya, gxa = _step(a, _x(4))
    yb, gxb = _step(b, _x(4))
    torch.cuda.synchronize()
    assert torch.equal(ya, yb) and torch.equal(gxa, gxb)
    _assert_same_grads(_grads(a), _grads(b), "step 2")


def test_gradient_accumulation_two_micro_batches():
    """Two forward / backward passes accumulate into .grad before one optimizer step
    (yolov8_qat.py:257-260, `accumulate`)."""
    a, b = _pair()
    for m in (a, b):
        for s in (5, 6):
            m(_x(s)).square().mean().backward()
    torch.cuda.synchronize()
    _assert_same_grads(_grads(a), _grads(b), "accumulated")
    assert D.pending_count() == 0


def test_deep_copy_ema_equals_per_call():
    """ModelEMA's deepcopy (utils/util.py:386) of a model in the learning phase: the copy
    carries its own launch hooks (fresh caches), its eval forward equals the per-call
    model's, and a training step on the copy equals the per-call path too."""
    a, b = _pair()
    ea, eb = copy.deepcopy(a).eval(), copy.deepcopy(b).eval()
    assert V.model_launches_enabled(ea) and not V.model_launches_enabled(eb)
    x = _x(7)
    with torch.no_grad():
        assert torch.equal(ea(x), eb(x))
    ea.train(), eb.train()
    ya, gxa = _step(ea, x)
    yb, gxb = _step(eb, x)
    torch.cuda.synchronize()
    assert torch.equal(ya, yb) and torch.equal(gxa, gxb)
    _assert_same_grads(_grads(ea), _grads(eb), "copy")
    assert not _grads(a)   # the original saw nothing of the copy's step


def test_graphed_step_equals_per_call_eager():
    from vsiquantization_amd.utils.graph import GraphedStep
    a, b = _pair()
    x = _x(8)
    params = [p for p in a.parameters() if p.requires_grad]

    def step():
        y = a(x)
        y.square().mean().backward()
        return y

    gs = GraphedStep(step, grads_of=params)
    for _ in range(3):
        y = gs()
    torch.cuda.synchronize()
    yb, _ = _step(b, x)
    torch.cuda.synchronize()
    assert torch.equal(y, yb)
    _assert_same_grads(_grads(a), _grads(b), "graph")


def test_state_dict_round_trip(tmp_path):
    """torch.save(state_dict) after a step (yolov8_qat.py:299) and load_partial_checkpoint
    into a fresh model from the same sequence: identical parameters (f64 scales by name)
    and an identical next step on either path."""
    a = _model()
    _step(a, _x(9))
    torch.optim.SGD(a.parameters(), lr=1e-2).step()
    path = tmp_path / "last_qat.pth"
    torch.save(a.state_dict(), path)
    c = _model()
    assert load_partial_checkpoint(c, str(path)) == len(a.state_dict())
    for (n, p), (n2, q) in zip(a.state_dict().items(), c.state_dict().items()):
        assert n == n2 and torch.equal(p, q), n
    assert c.state_dict()["0.weight_quantizer.scale"].dtype == torch.float64
    a.zero_grad(set_to_none=True)
    ya, _ = _step(a, _x(10))
    yc, _ = _step(c, _x(10))
    torch.cuda.synchronize()
    assert torch.equal(ya, yc)
    _assert_same_grads(_grads(a), _grads(c), "reloaded")


def test_whole_model_pickles_with_its_hooks(tmp_path):
    """The launch hooks are objects, not closures: a whole-model torch.save / load (not the
    reference's state_dict flow, but common) keeps them and gives the same step."""
    a = _model()
    path = tmp_path / "model.pt"
    torch.save(a, path)
    c = torch.load(path, weights_only=False)   # our own file (written just above)
    assert V.model_launches_enabled(c)
    ya, _ = _step(a, _x(11))
    yc, _ = _step(c, _x(11))
    torch.cuda.synchronize()
    assert torch.equal(ya, yc)


def test_opt_outs(monkeypatch):
    monkeypatch.setenv("VSIQ_MODEL_LAUNCHES", "0")
    m = _model()
    assert not V.model_launches_enabled(m)
    monkeypatch.delenv("VSIQ_MODEL_LAUNCHES")
    m = _model()
    assert V.model_launches_enabled(m)
    V.disable_model_launches(m)
    assert not V.model_launches_enabled(m) and not m._forward_hooks
    V.enable_model_launches(m)
    V.enable_model_launches(m)   # idempotent
    assert len(m._forward_pre_hooks) == 2 and len(m._forward_hooks) == 1


def test_quantizer_off_weight_stays_unquantized():
    """deactivate_quantizer on a layer (is_quantize False, qm.py:86-90 returns the weight
    as is): K7 must not hand that layer a fake-quantized weight."""
    from vsiquantization_amd.utils.quantize_manager import deactivate_quantizer
    a, b = _pair()
    for m in (a, b):
        deactivate_quantizer(m, layer_names=["1"])
    x = _x(12)
    ya, gxa = _step(a, x)
    yb, gxb = _step(b, x)
    torch.cuda.synchronize()
    assert torch.equal(ya, yb) and torch.equal(gxa, gxb)


def test_symmetric_tensor_zero_point_stays_per_call():
    """A symmetric quantizer handed a gradient-requiring tensor zero point (K4 zp_learn 2:
    zp used as given) is left out of K7 / K4d and gives the per-call path's results,
    including the zero point's gradient."""
    a, b = _pair()
    for m in (a, b):
        for layer in m:
            for qm in (layer.weight_quantizer, layer.activation_quantizer):
                if qm.quantizer.symmetric:
                    qm.zero_point = nn.Parameter(torch.tensor(0.25, dtype=torch.float64, device=DEV))
    x = _x(13)
    ya, gxa = _step(a, x)
    yb, gxb = _step(b, x)
    torch.cuda.synchronize()
    assert torch.equal(ya, yb) and torch.equal(gxa, gxb)
    ga, gb = _grads(a), _grads(b)
    assert any(n.endswith("weight_quantizer.zero_point") for n in ga)
    _assert_same_grads(ga, gb, "sym tensor zp")
    assert D.pending_count() == 0
