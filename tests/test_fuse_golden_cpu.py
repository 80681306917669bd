"""fuse_modules_unified against the structure the REFERENCE produced on the same toy
model and FuseConfigManager (tests/golden/gen_goldens.py §9; modules/fuse.py:45-149,
fuse_config.py:57-149): which children fuse into which class, which config each fused
layer got -- looked up by the CHILD name of its first module (fuse.py:113-114), so the
path pattern "stem" never matches and "^conv$" does -- and the BN fold on the host
(fused.py:100-108) within one ulp of the reference's (torch CPU ops on another CPU may
vectorize differently; the GPU fold is checked bitwise in test_gpu_fused_golden.py).
CPU only: construction does not launch kernels."""
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn

from vsiquantization_amd.modules.fuse import fuse_modules_unified
from vsiquantization_amd.modules.fuse_config import FuseConfig, FuseConfigManager
from tests import goldens as G


def toy_model():
    """The generator's toy model (same modules, same order); weights from the fixture."""
    return nn.Sequential(OrderedDict(
        stem=nn.Sequential(OrderedDict(conv=nn.Conv2d(3, 8, 3, padding=1, bias=False),
                                       bn=nn.BatchNorm2d(8), act=nn.ReLU())),
        block=nn.Sequential(OrderedDict(conv1=nn.Conv2d(8, 8, 1), relu1=nn.SiLU(),
                                        conv2=nn.Conv2d(8, 16, 3, padding=1, bias=False),
                                        bn2=nn.BatchNorm2d(16))),
        tail=nn.Sequential(nn.Conv2d(16, 16, 3, padding=1), nn.ReLU(), nn.Conv2d(16, 4, 1)),
        head=nn.Sequential(OrderedDict(pool=nn.Flatten(), fc=nn.Linear(4 * 8 * 8, 10),
                                       bn=nn.BatchNorm1d(10), act=nn.ReLU())),
    ))


def _fused():
    case = G.cases("fuse_structure")[0]
    model = toy_model()
    model.load_state_dict({k: torch.from_numpy(G.arr(v)) for k, v in case["state_dict"].items()})
    cfgs = case["configs"]
    cm = FuseConfigManager(FuseConfig(**cfgs["default"]))
    for pat in ("stem", "^conv$", "conv2", "^0$", "fc"):
        cm.add_layer_config(pat, FuseConfig(**cfgs[pat]))
    return case, fuse_modules_unified(model, case["patterns"], is_trace=False, config_manager=cm)


def test_fuse_structure_matches_reference():
    case, model = _fused()
    got = []
    for name, mod in model.named_modules():
        ent = dict(name=name, type=type(mod).__name__)
        if hasattr(mod, "weight_quantizer"):
            ent.update(bits_w=mod.bits_w, bits_a=mod.bits_a,
                       w_sym=mod.weight_quantizer.quantizer.symmetric,
                       a_sym=mod.activation_quantizer.quantizer.symmetric,
                       qw=type(mod.weight_quantizer.quantizer).__name__,
                       ow=type(mod.weight_quantizer.observer).__name__,
                       is_fuse_bn=getattr(mod, "is_fuse_bn", None), has_bn=hasattr(mod, "bn"),
                       is_relu=getattr(mod, "is_relu", None))
        got.append(ent)
    assert got == case["structure"]


def test_host_fold_within_one_ulp_of_reference():
    case, model = _fused()
    ref = toy_model()
    ref.load_state_dict({k: torch.from_numpy(G.arr(v)) for k, v in case["state_dict"].items()})
    for path, core_name in (("stem.conv", "conv_fuse"), ("head.fc", "linear_fuse")):
        m = model.get_submodule(path)
        core = getattr(m, core_name)
        src = ref.get_submodule(path)
        bn = ref.get_submodule(path.rsplit(".", 1)[0] + ".bn")
        std = np.sqrt(bn.running_var.numpy().astype(np.float64) + bn.eps)
        scale = bn.weight.detach().numpy().astype(np.float64) / std
        want = src.weight.detach().numpy().astype(np.float64) * scale.reshape([-1] + [1] * (src.weight.dim() - 1))
        np.testing.assert_allclose(core.weight.detach().numpy(), want, rtol=3e-7, atol=1e-30)
