"""End-to-end QAT training step of a YOLOv8n-backbone-shaped conv chain on one MI355X
(experiment): the model a reference user builds -- Conv+BN+ReLU layers swapped for fused
ConvBnReLU QAT layers, calibrated, learnable f64 scales activated (yolov8_qat.py:86-92,
utils/quantize_manager.py) -- trained with forward + backward + SGD step, in four forms:

  float      the same chain without fake quant (folded BN, conv + ReLU): the floor
  reference  the reference's algorithm as eager torch on the same GPU: per layer the
             learnable weight fake quant and the activation fake quant of uniform.py:47-56
             (x / s + zp, RoundStraightThrough, clamp, (q - zp) * s, ScaleGradient), the
             fused layer's conv -> ReLU -> quantize_out (modules/fused.py:112-134)
  per-call   vsiquantization_amd's fused layers on the per-call path (K5 act fake quant with
             the ReLU fused, K1/K4 weight fake quant, C++ autograd nodes; model_launches=False)
  default    the reference's plain sequence (calibrate_qat_model, activate_learning_qparam,
             activate_quantizer), which since round 4 installs the model-level launches by
             itself: K7 (one weight launch each way) and K4d (records + one fold launch)

The 27 layers take the backbone's (cout, k, stride) in forward order with cin chained
(the CSP concats are not modelled), 320x320 input, w2/a4 symmetric (the YAML default).
Prints ms per training step (median of 5 runs of STEPS steps) and the first step's loss
of each quantized form (the same algorithm: equal up to conv / reduction order)."""
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vsiquantization_amd.modules.fused import ConvBnReLU  # noqa: E402
from vsiquantization_amd.utils.quantize_manager import (activate_learning_qparam, activate_quantizer,  # noqa: E402
                                                        calibrate_qat_model, data_calib)

dev = torch.device(os.environ.get("DEV", "cuda:0"))
BATCH = int(os.environ.get("BATCH", "32"))
STEPS = int(os.environ.get("STEPS", "10"))
BITS_W, BITS_A = 2, 4


def chain(seed=0):
    torch.manual_seed(seed)
    mods, c = [], 3
    for _, cout, k, s, _ in bench.yolov8n_backbone():
        conv = nn.Conv2d(c, cout, k, s, padding=(k - 1) // 2, bias=False)
        bn = nn.BatchNorm2d(cout, eps=1e-3)
        bn.running_mean.uniform_(-0.1, 0.1)
        bn.running_var.uniform_(0.5, 2.0)
        mods.append((conv, bn))
        c = cout
    return mods


def ours(mods, launches=None):
    m = nn.Sequential(*[ConvBnReLU(cv, bn, nn.ReLU(), "MinMaxObserver", "UniformQuantizer", "MinMaxObserver",
                                   "UniformQuantizer", True, True, True, BITS_W, BITS_A) for cv, bn in mods]).to(dev)
    g = torch.Generator().manual_seed(5)
    loader = [(torch.randint(0, 256, (8, 3, 320, 320), generator=g, dtype=torch.uint8), None) for _ in range(2)]
    calibrate_qat_model(m, loader, data_calib, dev)
    activate_learning_qparam(m, model_launches=launches)
    activate_quantizer(m, model_launches=launches)
    return m.train()


class RoundSTE(torch.autograd.Function):          # uniform.py:258-271
    @staticmethod
    def forward(ctx, x):
        return torch.round(x)

    @staticmethod
    def backward(ctx, g):
        return g


class ScaleGradient(torch.autograd.Function):     # uniform.py:242-255
    @staticmethod
    def forward(ctx, x, scale):
        ctx.scale = scale
        return x

    @staticmethod
    def backward(ctx, g):
        return g * ctx.scale, None


def fq_learn(x, scale, bits):                     # uniform.py:47-56, symmetric (zp = 0)
    qmin, qmax = -(2 ** (bits - 1)), 2 ** (bits - 1) - 1
    s = ScaleGradient.apply(scale, (qmax * x.numel()) ** -0.5)
    x_int = torch.clamp(RoundSTE.apply(x / s + 0), qmin, qmax)
    return (x_int - 0) * s


class RefLayer(nn.Module):
    """The reference's fused layer in the learning phase, eager torch (fused.py:112-134)."""

    def __init__(self, layer, quantize):
        super().__init__()
        cv = layer.conv_fuse
        self.weight = nn.Parameter(cv.weight.detach().clone())
        self.bias = nn.Parameter(cv.bias.detach().clone()) if cv.bias is not None else None
        self.stride, self.padding = cv.stride, cv.padding
        self.quantize = quantize
        if quantize:
            self.sw = nn.Parameter(layer.weight_quantizer.scale.detach().clone())
            self.sa = nn.Parameter(layer.activation_quantizer.scale.detach().clone())

    def forward(self, x):
        w = fq_learn(self.weight, self.sw, BITS_W) if self.quantize else self.weight
        y = F.relu(F.conv2d(x, w, self.bias, self.stride, self.padding))
        return fq_learn(y, self.sa, BITS_A) if self.quantize else y


def step_fn(m, x):
    opt = torch.optim.SGD(m.parameters(), lr=1e-6)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = m(x).mean()
        loss.backward()
        opt.step()
        return loss
    return step


def timed(step):
    first = float(step().detach())
    for _ in range(2):
        step()
    res = []
    for _ in range(5):
        torch.cuda.synchronize() if dev.type == "cuda" else None
        t0 = time.perf_counter()
        for _ in range(STEPS):
            step()
        torch.cuda.synchronize() if dev.type == "cuda" else None
        res.append((time.perf_counter() - t0) / STEPS * 1e3)
    return sorted(res)[2], first


def main():
    x = (torch.randint(0, 256, (BATCH, 3, 320, 320), generator=torch.Generator().manual_seed(9),
                       dtype=torch.uint8).float() / 255).to(dev)
    want = os.environ.get("VARIANTS", "float,reference,ours,plus").split(",")
    base = ours(chain(), launches=False)
    rows = {}
    if "float" in want:
        rows["float"] = timed(step_fn(nn.Sequential(*[RefLayer(l, False) for l in base]).to(dev), x))
    if "reference" in want:
        rows["reference (eager torch)"] = timed(step_fn(nn.Sequential(*[RefLayer(l, True) for l in base]).to(dev),
                                                        x))
    if "ours" in want:
        rows["ours, per-call path"] = timed(step_fn(base, x))
    if "plus" in want:
        plus = ours(chain())   # the reference sequence: K7 + K4d installed by activate_*
        rows["ours, default (K7 + K4d)"] = timed(step_fn(plus, x))
    print(f"batch {BATCH}, 27 layers, 320x320, w{BITS_W}/a{BITS_A}; ms per training step (fwd + bwd + SGD)")
    fl = rows["float"][0] if "float" in rows else 0.0
    for k, (ms, loss) in rows.items():
        print(f"{k:34s} {ms:8.2f} ms   QAT overhead over float {ms - fl:7.2f} ms   first loss {loss:.6f}",
              flush=True)


if __name__ == "__main__":
    main()
