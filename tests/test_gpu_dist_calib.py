"""Batch-sharded calibration through the kernels, 2 ranks: per-tensor
activation observers (QuantizationManager, fused ReLU) with an all-reduce of their
statistics -- per call (K2 + finalize) and deferred (K2p records + one sync_calibration)
-- give the 1-GPU min/max and qparams bit for bit and mean|x| / mean / std within 1e-6
(observers/minmax.py:32-74, quantization_manager.py:55-71), including a call whose NaN
sits on one rank only; the 1-GPU run itself equals the oracle (observe_minmax /
minmax_qparams replayed call by call: bitwise; collect_stats: 1e-6).  Configurations
(tests/dist_calib_common.py): "small" (3 layers x 5 calls) and "c5" (C5's structure: the
27 backbone activation quantizers with ReLU x 16 calls of uint8/255-derived inputs, at 4
images per call).  The ranks run as a child torch.distributed.run job (gloo, both on
cuda:0: the collective is RCCL on a real multi-GPU node, the arithmetic around it is
the same).  test_c5_one_batch_full_size: one calibration batch of C5's 128 images per
GPU through the 27 deferred observers against the oracle."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import fakequant_np as O
from tests.dist_calib_common import DEV, Config, activations, managers, observe, state

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle(cfg, acts):
    """Per layer: the reference observer replayed over the calls (minmax.py:32-74, the
    manager's observer is 8-bit symmetric: SURVEY §0.5) and the per-call statistics."""
    out = []
    for li, (act, _) in enumerate(cfg.layers):
        mn, mx, stats = 0, 0, []
        for row in acts:
            a = O.act_forward(row[li].cpu().numpy(), act)
            mn, mx = O.observe_minmax(a, mn, mx)
            stats.append(O.collect_stats(a))
        s, z = O.minmax_qparams(mn, mx, True, 8)
        out.append(dict(min=float(mn), max=float(mx), scale=float(s), zp=float(z),
                        mean_abs=[t[0] for t in stats], mean=[t[1] for t in stats], std=[t[2] for t in stats]))
    return out


def _same(got, want, what):
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert (g["min"], g["max"], g["scale"], g["zp"]) == (w["min"], w["max"], w["scale"], w["zp"]), (what, i)
        for k in ("mean_abs", "mean", "std"):
            np.testing.assert_allclose(g[k], w[k], rtol=1e-6, atol=1e-12, err_msg=f"{what} layer {i} {k}")


@pytest.mark.parametrize("name", ["small", "c5"])
def test_sharded_calibration_two_ranks_equals_one_gpu(tmp_path, name):
    cfg = Config(name)
    out = tmp_path / "rank0.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_calib_worker.py"), str(out), name]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = json.loads(out.read_text())
    acts = activations(cfg)
    mgrs = managers(cfg)
    observe(cfg, mgrs, acts)
    one = state(mgrs)
    assert len(one[0]["mean_abs"]) == cfg.calls and len(one) == len(cfg.layers)
    _same(one, _oracle(cfg, acts), "1 GPU vs oracle")
    for mode in ("per_call", "deferred"):
        _same(got[mode], one, f"2 ranks {mode} vs 1 GPU")


def test_c5_one_batch_full_size():
    """C5 per GPU: one calibration batch of 128 images (3x320x320 network input; 274M
    activation elements over the 27 layers) through the deferred observers
    (calibrate_qat_model's default path: K2p + one sync) against the oracle."""
    import bench
    from vsiquantization_amd.distributed import sync_calibration
    cfg = Config("c5")
    cfg.calls, cfg.batch = 1, 128
    gen = torch.Generator(device=DEV)
    acts = [[]]
    for li, (_, shp) in enumerate(cfg.layers):
        gen.manual_seed(77 + li)
        u8 = torch.randint(0, 256, (cfg.batch, *shp), device=DEV, dtype=torch.uint8, generator=gen)
        acts[0].append((u8.float() / 255.0 - 0.45) * (0.5 + 0.25 * (li % 7)))
    assert sum(a.numel() for a in acts[0]) == 128 * 2_137_600 == 128 * sum(
        co * h * h for _, co, _, _, h in bench.yolov8n_backbone())
    mgrs = managers(cfg)
    for qm in mgrs:
        qm.dist_defer = True
    observe(cfg, mgrs, acts)
    sync_calibration(torch.nn.ModuleList(mgrs))
    _same(state(mgrs), _oracle(cfg, acts), "C5 batch 128 vs oracle")
