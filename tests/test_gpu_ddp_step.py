"""A 2-rank DistributedDataParallel QAT step over the learnable quantizers (SURVEY §8e;
reference: yolov8_qat.py:141-144 DDP, :239-263 backward + the f64 scale parameters;
quantizers/uniform.py:58-71 gscale from the LOCAL numel): the f64 scale / zero-point
gradients after DDP's all-reduce equal the average of the two ranks' local gradients
computed on one GPU (same shapes, same kernels, an average of two: bitwise in most runs,
within 1e-4 where MIOpen picked another conv algorithm in the other process), and the
activation scales carry the reference's local-numel ScaleGradient factor -- against the
full-batch 1-GPU step they are scaled by sqrt(world)/world, the weight scales by
1/world (within the conv's rounding differences between batch shapes).  The ranks run as a child torch.distributed.run job
(gloo, both on cuda:0)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

from tests.ddp_common import batch, model, quant_grads

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("deferred", [False, True, "default"])
def test_ddp_learnable_step_two_ranks(tmp_path, deferred):
    """deferred: the ranks run enable_deferred_qparam_grads (records-only K4 + one fold at the
    end of the backward, quantizers/deferred.py): DDP's hooks see the folded gradients.
    "default": the model-level launches activate_learning_qparam / activate_quantizer
    install by themselves (K7 weights + K4d), the reference's own sequence."""
    out = tmp_path / "grads.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "ddp_step_worker.py"), str(out)]
    env = dict(os.environ, VSIQ_TEST_DEFERRED=deferred if isinstance(deferred, str) else ("1" if deferred else "0"))
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = json.loads(out.read_text())
    dtypes = got.pop("_dtypes")
    # one GPU: each rank's local step, then the average DDP computes
    m = model()
    x = batch()
    local = []
    for part in x.chunk(2):
        m.zero_grad(set_to_none=True)
        m(part).square().sum().backward()
        local.append(quant_grads(m))
    assert set(got) == set(local[0])
    scales = [n for n in got if n.endswith("scale") or n.endswith("zero_point")]
    assert len(scales) == 5 and all(dtypes[n] == "torch.float64" for n in scales)
    rel = {}
    for n in got:
        want = (local[0][n] + local[1][n]) / 2
        g = torch.tensor([float.fromhex(v) for v in got[n]], dtype=torch.float64).reshape(want.shape)
        d = (g - want.double().cpu()).abs().max() / want.double().abs().max().clamp_min(1e-30)
        rel[n] = float(d)
    print(rel)
    # same kernels and shapes on both sides, but the convs are MIOpen's in another process,
    # which may select another algorithm (bitwise equal in most runs; scale gradients are
    # sums with heavy cancellation, so a last-bit conv difference shows up larger there)
    assert all(v <= (1e-4 if n.endswith(("scale", "zero_point")) else 1e-5) for n, v in rel.items()), rel
    # against the full-batch step: activation scales x sqrt(2)/2 (local numel), weights' the same
    m.zero_grad(set_to_none=True)
    m(x).square().sum().backward()
    full = quant_grads(m)
    for n in scales:
        ddp = float.fromhex(got[n][0])
        f = float(full[n])
        # with a sum loss the ranks' gradient sums add up to the full batch's and DDP's
        # average halves them; an activation quantizer's gscale (qmax * local numel)^-1/2 is
        # sqrt(2) x the full batch's, a weight quantizer's is the same on every rank
        want = f * ((2 ** 0.5) / 2 if "activation_quantizer" in n else 0.5)
        assert abs(ddp - want) <= 2e-3 * abs(want), (n, ddp, want)
