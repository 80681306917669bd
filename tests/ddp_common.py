"""Model, data and gradient extraction shared by tests/test_gpu_ddp_step.py and its
worker (tests/ddp_step_worker.py): a two-layer fused QAT model in the learning phase --
calibrated on every rank with the same loader (the reference does not shard its
calibration, yolov8_qat.py:86-92), learnable f64 scales (qm.py:92-114), the second
layer's activation quantizer an asymmetric LSQQuantizer with a learnable zero point."""
import torch
import torch.nn as nn

from vsiquantization_amd.modules.fused import ConvBnReLU
from vsiquantization_amd.utils.quantize_manager import (activate_learning_qparam, activate_quantizer,
                                                        calibrate_qat_model, data_calib)

DEV = "cuda:0"
BATCH = 4


def _bn(c, seed):
    torch.manual_seed(seed)
    bn = nn.BatchNorm2d(c, eps=1e-3)
    bn.running_mean.uniform_(-0.3, 0.3)
    bn.running_var.uniform_(0.2, 3.0)
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.uniform_(-0.2, 0.2)
    return bn


def model(launches=False):
    """launches: the model-level launches (K7 + K4d) that activate_learning_qparam /
    activate_quantizer install by default; False: the per-call path."""
    # MIOpen's default weight-gradient kernels may accumulate with atomics: deterministic
    # algorithms, so the ranks' conv gradients do not differ from run to run
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    torch.manual_seed(0)
    a = ConvBnReLU(nn.Conv2d(3, 8, 3, padding=1, bias=False), _bn(8, 1), nn.ReLU(), "MinMaxObserver",
                   "UniformQuantizer", "MinMaxObserver", "UniformQuantizer", True, True, True, 4, 4)
    b = ConvBnReLU(nn.Conv2d(8, 16, 3, padding=1, bias=False), _bn(16, 2), nn.ReLU(), "MinMaxObserver",
                   "UniformQuantizer", "MinMaxObserver", "LSQQuantizer", True, False, True, 8, 8)
    m = nn.Sequential(a, b).to(DEV)
    g = torch.Generator().manual_seed(5)
    loader = [(torch.randint(0, 256, (2, 3, 16, 16), generator=g, dtype=torch.uint8), None) for _ in range(3)]
    calibrate_qat_model(m, loader, data_calib, DEV)
    activate_learning_qparam(m, model_launches=launches)
    activate_quantizer(m, model_launches=launches)
    m.train()
    return m


def batch():
    g = torch.Generator().manual_seed(9)
    return (torch.randint(0, 256, (BATCH, 3, 16, 16), generator=g, dtype=torch.uint8).float() / 255).to(DEV)


def quant_grads(m):
    """name -> gradient (f64 for the learnable scales / zero points; conv weights fp32)."""
    return {n: p.grad.detach().clone() for n, p in m.named_parameters()
            if p.grad is not None and (n.endswith("scale") or n.endswith("zero_point") or n.endswith("weight"))}
