"""bench.py's N > 1 act leg under HIP-graph capture: a 1-rank RCCL group drives
bench.ActQuant with its per-call exchange (per layer: K2 records, RCCL
all_gather_into_tensor, K1r fold + fake quant) through capture_groups and replay --
bit-identical to direct launches -- and through measure(), which reports its launch
mode.  (RCCL cannot put two ranks on one GPU; the driver's 8-GPU run is the N > 1
case.)  Reference: yolov8_qat.py:423-429 / 134-144 (DDP), observers/minmax.py:42-47."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_act_leg_graph_capture_with_rccl_exchange():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "bench_capture_worker.py")]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    why = [l for l in r.stderr.splitlines() if "terminated with exception" in l or "Error" in l][:6]
    assert r.returncode == 0, "\n".join(why) + r.stdout[-2000:] + r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    got = json.loads(line)
    assert got["graph_equals_direct"] and got["self_check"], got
    # the captured all_gathers ran on the world's capture-only twin
    assert got["capture_twin"] and got["world_after"] == 1.0, got
    assert got["launch"] in ("direct", "hip graph per phase and group") and got["alt"] is not None, got
