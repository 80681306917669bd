"""Model, loader and state extraction shared by tests/test_gpu_dist_calib.py and its
worker (tests/dist_calib_worker.py)."""
import torch
import torch.nn as nn

from vsiquantization_amd.modules.fused import ConvBnReLU

DEV = "cuda:0"


def model():
    torch.manual_seed(0)
    layers = []
    for cin, cout in ((3, 16), (16, 32), (32, 32)):
        cv = nn.Conv2d(cin, cout, 3, padding=1, bias=False)
        bn = nn.BatchNorm2d(cout)
        bn.running_var.uniform_(0.5, 2.0)
        layers.append(ConvBnReLU(cv, bn, nn.ReLU(), "MinMaxObserver", "UniformQuantizer", "MinMaxObserver",
                                 "UniformQuantizer", True, True, True, 4, 4))
    return nn.Sequential(*layers).to(DEV)


def loader(n=5):
    g = torch.Generator().manual_seed(3)
    return [(torch.randint(0, 256, (4, 3, 24, 24), generator=g, dtype=torch.uint8), None) for _ in range(n)]


def state(m):
    """Per activation manager: observer min/max, f64 qparams and the mean|x| / mean / std
    lists (quantization_manager.py:55-71)."""
    out = []
    for layer in m:
        qm = layer.activation_quantizer
        out.append(dict(min=float(qm.observer.min_val), max=float(qm.observer.max_val),
                        scale=float(qm.scale), zp=float(qm.zero_point),
                        mean_abs=[float(v) for v in qm.mean_abs_x], mean=[float(v) for v in qm.mean_x],
                        std=[float(v) for v in qm.std]))
    return out
