"""Activations, managers and state extraction shared by the sharded-calibration GPU tests
(tests/test_gpu_dist_calib.py) and their worker (tests/dist_calib_worker.py).

Two configurations:
* "small": 3 layers (ReLU / none / ReLU) x 5 calls of [4, 8, 10, 10];
* "c5": C5's structure -- the YOLOv8n backbone's 27 activation quantizers, all with
  the fused ReLU (modules/fused.py:133), 16 calibration calls (yolov8_qat.py:42-52
  breaks after batch 15) -- at a reduced batch of 4 images per call, the activations
  derived from uint8 images / 255 (yolov8_qat.py:47) by a per-layer affine map.

The observed tensors are generated directly (seeded, identically in every process), not
by a conv: a conv's fp32 result may depend on the batch size (MIOpen picks its
algorithm per shape), which would test MIOpen, not the observer exchange."""
import numpy as np
import torch

from vsiquantization_amd.quantizers.quantization_manager import QuantizationManager

DEV = "cuda:0"


def _backbone():
    import bench
    return bench.yolov8n_backbone()


class Config:
    def __init__(self, name):
        self.name = name
        if name == "small":
            self.layers = [("relu", (8, 10, 10)), (None, (8, 10, 10)), ("relu", (8, 10, 10)), ("silu", (8, 12, 10))]
            self.calls, self.batch, self.nan_at = 5, 4, (2, 1)
        elif name == "c5":
            self.layers = [("relu", (co, h, h)) for _, co, _, _, h in _backbone()]
            self.calls, self.batch, self.nan_at = 16, 4, (9, 20)
        else:
            raise ValueError(name)


def activations(cfg):
    """[call][layer] -> float32 [batch, ...] on the device; one NaN in the LAST image of
    call/layer cfg.nan_at (on one rank only when sharded), which the whole call must skip
    (observers/minmax.py:42-47: Python's < is False against NaN)."""
    out = []
    if cfg.name == "small":
        rng = np.random.default_rng(7)
        scales = (1.0, 0.3, 4.0, 2.0)
        for c in range(cfg.calls):
            row = []
            for li, (_, shp) in enumerate(cfg.layers):
                a = (rng.standard_normal((cfg.batch, *shp)) * scales[li] * (1 + 0.3 * c)).astype(np.float32)
                row.append(torch.from_numpy(a).to(DEV))
            out.append(row)
    else:
        gen = torch.Generator(device=DEV)
        for c in range(cfg.calls):
            row = []
            for li, (_, shp) in enumerate(cfg.layers):
                gen.manual_seed(1000 * c + li)
                u8 = torch.randint(0, 256, (cfg.batch, *shp), device=DEV, dtype=torch.uint8, generator=gen)
                gain = 0.5 + 0.25 * (li % 7) + 0.05 * c
                row.append((u8.float() / 255.0 - 0.45) * gain)
            out.append(row)
    c, li = cfg.nan_at
    out[c][li].view(cfg.batch, -1)[cfg.batch - 1, 17] = float("nan")
    return out


def managers(cfg):
    mgrs = []
    for _ in cfg.layers:
        qm = QuantizationManager("UniformQuantizer", "MinMaxObserver", 4, True, is_learning_scale=False)
        qm.is_observer_qparam, qm.is_quantize = True, False
        mgrs.append(qm.to(DEV))
    return mgrs


def observe(cfg, mgrs, acts, shard=None):
    """Every call of every layer through QuantizationManager.quantize (qm.py:73-90);
    shard = (rank, world) observes that rank's part of each batch."""
    for row in acts:
        for qm, x, (act, _) in zip(mgrs, row, cfg.layers):
            if shard is not None:
                x = x.chunk(shard[1])[shard[0]]
            qm.quantize(x, act=act)


def observe_quantize(cfg, mgrs, acts, shard=None):
    """Observe + quantize mode (qm.py:73-90 with is_quantize): every call's
    y and its straight-through gradient of a seeded upstream gradient, per (call, layer);
    shard = (rank, world): that rank's part of each batch (and of each gradient)."""
    out = {}
    for c, row in enumerate(acts):
        for li, (qm, x, (act, _)) in enumerate(zip(mgrs, row, cfg.layers)):
            gen = torch.Generator(device=DEV).manual_seed(50_000 + 100 * c + li)
            g = torch.randn(x.shape, device=DEV, generator=gen)
            if shard is not None:
                x, g = x.chunk(shard[1])[shard[0]], g.chunk(shard[1])[shard[0]]
            xr = x.clone().requires_grad_(True)
            y = qm.quantize(xr, act=act)
            y.backward(g)
            out[f"y{c}_{li}"] = y.detach().cpu().numpy()
            out[f"g{c}_{li}"] = xr.grad.cpu().numpy()
    return out


def state(mgrs):
    """Per manager: observer min/max, qparams and the mean|x| / mean / std lists
    (quantization_manager.py:55-71)."""
    out = []
    for qm in mgrs:
        out.append(dict(min=float(qm.observer.min_val), max=float(qm.observer.max_val),
                        scale=float(qm.scale), zp=float(qm.zero_point),
                        mean_abs=[float(v) for v in qm.mean_abs_x], mean=[float(v) for v in qm.mean_x],
                        std=[float(v) for v in qm.std]))
    return out
