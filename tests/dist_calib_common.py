"""Activations, managers and state extraction shared by tests/test_gpu_dist_calib.py and
its worker (tests/dist_calib_worker.py).  The observed tensors are generated directly
(seeded), not by a conv: a conv's fp32 result may depend on the batch size (MIOpen
picks its algorithm per shape), which would test MIOpen, not the observer exchange."""
import numpy as np
import torch

from vsiquantization_amd.quantizers.quantization_manager import QuantizationManager

DEV = "cuda:0"
LAYERS = (("relu", 1.0), (None, 0.3), ("relu", 4.0))
CALLS = 5
BATCH = 4


def activations():
    """[call][layer] -> float32 [BATCH, 8, 10, 10] on the device (one NaN-free batch each;
    layer 1 of call 2 holds a NaN in its second half, which the whole call must skip)."""
    rng = np.random.default_rng(7)
    out = []
    for c in range(CALLS):
        row = []
        for li, (_, scale) in enumerate(LAYERS):
            a = (rng.standard_normal((BATCH, 8, 10, 10)) * scale * (1 + 0.3 * c)).astype(np.float32)
            if (c, li) == (2, 1):
                a[BATCH - 1, 3, 4, 5] = np.nan
            row.append(torch.from_numpy(a).to(DEV))
        out.append(row)
    return out


def managers():
    mgrs = []
    for _ in LAYERS:
        qm = QuantizationManager("UniformQuantizer", "MinMaxObserver", 4, True, is_learning_scale=False)
        qm.is_observer_qparam, qm.is_quantize = True, False
        mgrs.append(qm.to(DEV))
    return mgrs


def observe(mgrs, acts, shard=None):
    """Every call of every layer through QuantizationManager.quantize (qm.py:73-90);
    shard = (rank, world) observes that rank's part of each batch."""
    for row in acts:
        for qm, x, (act, _) in zip(mgrs, row, LAYERS):
            if shard is not None:
                x = x.chunk(shard[1])[shard[0]]
            qm.quantize(x, act=act)


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
