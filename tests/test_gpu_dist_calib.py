"""Batch-sharded calibration through the kernels, 2 ranks: per-tensor
activation observers (QuantizationManager, fused ReLU) with an all-reduce of their
statistics — per call (K2 + finalize) and deferred (K2p records + one sync_calibration)
— give the 1-GPU min/max and qparams bit for bit and mean|x| / mean / std within 1e-6
(observers/minmax.py:32-74, quantization_manager.py:55-71), including a call whose NaN
sits on one rank only.  The ranks run as a child torch.distributed.run job (gloo, both
on cuda:0: the collective is RCCL on a real multi-GPU node, the arithmetic around it is
the same)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from tests.dist_calib_common import activations, managers, observe, state

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_calibration_two_ranks_equals_one_gpu(tmp_path):
    out = tmp_path / "rank0.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_calib_worker.py"), str(out)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = json.loads(out.read_text())
    mgrs = managers()
    observe(mgrs, activations())
    want = state(mgrs)
    assert len(want[0]["mean_abs"]) == 5
    for mode in ("per_call", "deferred"):
        for g, w in zip(got[mode], want):
            assert (g["min"], g["max"], g["scale"], g["zp"]) == (w["min"], w["max"], w["scale"], w["zp"]), mode
            for k in ("mean_abs", "mean", "std"):
                np.testing.assert_allclose(g[k], w[k], rtol=1e-6, atol=1e-12, err_msg=f"{mode} {k}")
