"""Host-side API parity on CPU: registry, constructors, attributes, config resolution,
fusion structure, BN folding, lifecycle flags.  No kernel launches."""
import os

import pytest
import torch
import torch.nn as nn

import vsiquantization_amd as V
from vsiquantization_amd.modules import (ConvBn, ConvBnReLU, ConvReLU, FuseConfig, Linear, LinearBnReLU,
                                         LinearReLU, create_fuse_config_manager, fuse_modules_unified,
                                         load_fuse_config_from_yaml)
from vsiquantization_amd.modules.fuse import _fuse_modules_trace
from vsiquantization_amd.utils.quantize_manager import (activate_learning_qparam, activate_quantizer,
                                                        calibrate_qat_model, deactivate_quantizer)
from vsiquantization_amd.utils.registry import CLASS_REGISTRY, register_class

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_registry_names():
    for name in ("UniformQuantizer", "MinMaxObserver", "LSQQuantizer", "LSQObserver",
                 "PerChannelUniformQuantizer", "PerChannelMinMaxObserver"):
        assert name in CLASS_REGISTRY
    assert CLASS_REGISTRY["UniformQuantizer"] is V.UniformQuantizer

    @register_class
    class _Tmp:
        pass
    assert CLASS_REGISTRY.pop("_Tmp") is _Tmp


@pytest.mark.parametrize("bits,sym,lo,hi", [(8, True, -128, 127), (8, False, 0, 255), (4, True, -8, 7),
                                            (2, True, -2, 1), (2, False, 0, 3)])
def test_quantizer_ranges(bits, sym, lo, hi):
    q = CLASS_REGISTRY["UniformQuantizer"](bits, sym)   # positional, like qm.py:41
    assert (q.qmin, q.qmax, q.num_bits, q.symmetric, q.calib_grad_scale) == (lo, hi, bits, sym, 1)
    assert q.calculate_grad_scale(torch.empty(10, 10)) == (hi * 100) ** -0.5


def test_observer_host_semantics():
    o = CLASS_REGISTRY["MinMaxObserver"](False)           # positional, like qm.py:42
    assert (o.symmetric, o.num_bits, o.eps, o.min_val, o.max_val) == (False, 8, 1e-8, 0, 0)
    assert isinstance(o.min_val, int)
    o.min_val, o.max_val = -1.5, 2.5
    s, z = o.get_scale_zero_point()
    assert s == (2.5 - -1.5) / (255 + 1e-8) and z == round(1.5 / (s + 1e-8))
    o.min_val = float("-inf")
    with pytest.raises(ValueError):
        o.get_scale_zero_point()


def test_manager_attributes_and_quirks():
    qm = V.QuantizationManager("UniformQuantizer", "MinMaxObserver", 4, False)
    assert isinstance(qm, nn.Module)
    assert qm.is_symmetric is True                   # qm.py:50 hard-coded
    assert qm.quantizer.symmetric is False and qm.observer.symmetric is False
    assert qm.observer.num_bits == 8                 # observer built with is_symmetric only
    assert (qm.scale, qm.zero_point, qm.is_observer_qparam, qm.is_quantize) == (1, 0, True, True)
    assert qm.mean_abs_x == [] and qm.mean_x == [] and qm.std == []
    qm.mean_abs_x.extend([0.5, 1.5])
    qm.init_scaling_factor_for_learning()
    assert qm.scale == pytest.approx(2 * 1.0 / (7 ** 0.5))
    qm.make_learn_qparameter()
    assert isinstance(qm.scale, nn.Parameter) and qm.scale.dtype == torch.float64
    assert qm.zero_point == 0                        # UniformQuantizer never learns zp via manager
    assert "scale" in dict(qm.named_parameters())
    with pytest.raises(KeyError):
        V.QuantizationManager("NoSuchQuantizer", "MinMaxObserver", 8, True)


def test_lsq_manager_learns_zero_point():
    qm = V.QuantizationManager("LSQQuantizer", "LSQObserver", 8, False)
    qm.scale, qm.zero_point = 0.05, 128
    qm.make_learn_qparameter()
    assert isinstance(qm.zero_point, nn.Parameter) and qm.zero_point.dtype == torch.float64


def _toy():
    torch.manual_seed(0)
    m = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1, bias=False), nn.BatchNorm2d(8), nn.ReLU(),
                      nn.Conv2d(8, 8, 1), nn.BatchNorm2d(8), nn.SiLU(),
                      nn.Conv2d(8, 4, 3), nn.ReLU())
    for bn in (m[1], m[4]):
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.data.uniform_(0.5, 1.5)
        bn.bias.data.uniform_(-0.2, 0.2)
    return m


def test_fuse_structure_and_bn_fold():
    ref = _toy()
    m = _toy()
    cfg = load_fuse_config_from_yaml(os.path.join(ROOT, "vsiquantization_amd", "configs",
                                                  "fuse_config.yaml"))
    fuse_modules_unified(m, [["conv", "bn", "relu"], ["conv", "relu"]], is_trace=False, config_manager=cfg)
    assert isinstance(m[0], ConvBnReLU) and isinstance(m[1], nn.Identity) and isinstance(m[2], nn.Identity)
    assert isinstance(m[3], ConvBnReLU) and m[3].is_relu is False          # SiLU
    assert isinstance(m[6], ConvReLU) and isinstance(m[7], nn.Identity)
    # child-name config lookup quirk: child "0" matches no pattern -> default 2/4 bits
    assert (m[0].bits_w, m[0].bits_a) == (2, 4)
    assert m[0].weight_quantizer.quantizer.qmax == 1
    # BN fold (fused.py:100-108)
    std = torch.sqrt(ref[1].running_var + ref[1].eps)
    w = ref[0].weight * (ref[1].weight / std).reshape(-1, 1, 1, 1)
    b = ref[1].bias + (0 - ref[1].running_mean) * (ref[1].weight / std)
    assert torch.equal(m[0].conv_fuse.weight, w) and torch.equal(m[0].conv_fuse.bias, b)
    names = [n for n, _ in m.named_parameters()]
    assert "0.conv_fuse.weight" in names


def test_fuse_trace_mode_and_config_patterns():
    m = _toy()
    mgr = create_fuse_config_manager(FuseConfig(bits_w=8, bits_a=8),
                                     {"^3$": {"bits_w": 4, "bits_a": 4, "w_symmetric": False},
                                      "[": FuseConfig(bits_w=3)})   # invalid regex -> substring
    assert mgr.get_config_for_layer("3").bits_w == 4
    assert mgr.get_config_for_layer("x[y").bits_w == 3
    assert mgr.get_config_for_layer("zzz").bits_w == 8
    _fuse_modules_trace(m, [["conv", "bn", "relu"]], mgr)
    assert isinstance(m[0], ConvBnReLU) and isinstance(m[3], ConvBn) is False


def test_linear_layers_and_bias_handling():
    lin = nn.Linear(6, 5)
    bn = nn.BatchNorm1d(5)
    l1 = LinearBnReLU(lin, bn, nn.ReLU(), "MinMaxObserver", "UniformQuantizer", "MinMaxObserver",
                      "UniformQuantizer")
    assert l1.linear_fuse.bias is not None and l1.is_relu
    l2 = LinearReLU(lin, nn.SiLU(), "MinMaxObserver", "UniformQuantizer", "MinMaxObserver", "UniformQuantizer")
    assert torch.equal(l2.linear_fuse.bias, lin.bias) and l2.is_relu is False
    l3 = Linear(nn.Linear(6, 5, bias=False), "MinMaxObserver", "UniformQuantizer", "MinMaxObserver",
                "UniformQuantizer")
    assert l3.linear_fuse.bias is None


def test_lifecycle_flags():
    m = _toy()
    fuse_modules_unified(m, [["conv", "bn", "relu"]])
    seen = []
    calibrate_qat_model(m, None, lambda model, loader, dev: seen.append(model.training))
    assert seen == [False]
    for mod in m.modules():
        if hasattr(mod, "weight_quantizer"):
            for qm in (mod.weight_quantizer, mod.activation_quantizer):
                assert (qm.is_observer_qparam, qm.is_learning_scale, qm.is_quantize) == (True, False, False)
                qm.mean_abs_x = [0.1, 0.3]
    activate_learning_qparam(m, use_init=True)
    activate_quantizer(m)
    params = [n for n, _ in m.named_parameters() if n.endswith("scale")]
    assert "0.weight_quantizer.scale" in params and "0.activation_quantizer.scale" in params
    assert all(qm.is_quantize for mod in m.modules() if hasattr(mod, "weight_quantizer")
               for qm in (mod.weight_quantizer, mod.activation_quantizer))
    deactivate_quantizer(m, layer_names=["0"])
    assert m[0].weight_quantizer.is_quantize is False and m[3].weight_quantizer.is_quantize is True
    sd = m.state_dict()
    assert sd["0.weight_quantizer.scale"].dtype == torch.float64


def test_cpu_compute_runs_in_the_native_host_library(monkeypatch):
    """CPU tensors take the native host loops of the HIP library (vsiq_host_*), never the
    oracle: with the oracle unimportable the CPU path still runs."""
    import sys
    monkeypatch.setitem(sys.modules, "oracle", None)
    monkeypatch.setitem(sys.modules, "oracle.fakequant_np", None)
    q = V.UniformQuantizer(8, True)
    y = q.quantize(torch.tensor([0.0, 0.26, -1.0, 3.0]), 0.1, 0, False)
    assert y.tolist() == pytest.approx([0.0, 0.3, -1.0, 3.0])


def test_calib_grad_scale_factor_cached_per_tensor_version():
    """calib_grad_scale (utils/estimate_bn.py:136) may be a per-channel tensor: its sum is
    the effective ScaleGradient factor, read once per tensor / in-place version."""
    from vsiquantization_amd.quantizers.uniform import _calib_factor
    q = V.UniformQuantizer(8, True)
    assert _calib_factor(q) == 1.0
    c = torch.tensor([0.5, 0.25, 2.0])
    q.calib_grad_scale = c
    assert _calib_factor(q) == 2.75
    c.mul_(2.0)                                  # in-place: new version
    assert _calib_factor(q) == 5.5
    q.calib_grad_scale = torch.tensor([1.0, 1.0])
    assert _calib_factor(q) == 2.0
    q.calib_grad_scale = 0.5
    assert _calib_factor(q) == 0.5


def test_silu_layout_state_dict_round_trip():
    """QuantizationManager.silu_layout (the SiLU reference layout recorded with the qparams)
    travels in the state_dict only once recorded; strict loads work both ways (a checkpoint
    without it into a model that has none, and one with it into a fresh model)."""
    import torch.nn as nn
    from vsiquantization_amd import _hip as H
    mk = lambda: nn.Sequential(V.QuantizationManager("UniformQuantizer", "MinMaxObserver", 8, True))  # noqa: E731
    a = mk()
    assert "0.silu_layout" not in a.state_dict()
    assert a[0]._silu_act("silu").layout == H.silu_reference()
    assert a[0]._silu_act("relu") == "relu" and a[0]._silu_act(None) is None
    a[0].silu_layout = (32, 16)
    sd = a.state_dict()
    assert sd["0.silu_layout"].tolist() == [32, 16]
    b = mk()
    b.load_state_dict(sd)   # strict
    assert b[0].silu_layout == (32, 16)
    c = mk()
    c.load_state_dict(mk().state_dict())
    assert c[0].silu_layout is None
    act = b[0]._silu_act("silu") if H.silu_reference() == (32, 16) else None
    if act is None:
        import warnings
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            act = b[0]._silu_act("silu")
        assert any("SiLU reference layout" in str(x.message) for x in w)
    assert act == "silu" and act.layout == (32, 16) and H.act_code(act) == (H.ACT_SILU | (32 << 8) | (16 << 16))


def test_per_channel_observer_state_drops_its_bound_op():
    """The per-channel observer's cached C++ op (set by the public-API step on a GPU) is
    left out of its pickled / deep-copied state: copies rebuild their own."""
    import copy
    import pickle

    class Unpicklable:
        def __reduce__(self):
            raise TypeError("not picklable")

    obs = V.PerChannelMinMaxObserver(False)
    obs.observe(torch.randn(4, 6))
    obs._op = (obs.run_min, obs.run_max, (), Unpicklable())
    for c in (copy.deepcopy(obs), pickle.loads(pickle.dumps(obs))):
        assert "_op" not in c.__dict__
        assert torch.equal(c.run_min, obs.run_min) and torch.equal(c.scale, obs.scale)
    assert "_op" in obs.__dict__
