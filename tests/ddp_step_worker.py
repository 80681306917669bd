"""Worker of tests/test_gpu_ddp_step.py: one rank of a DistributedDataParallel QAT step
(torch.distributed.run, 2 ranks, gloo, both on cuda:0): DDP over the learnable model of
tests/ddp_common.py, each rank on its half of the batch, one backward (DDP's bucketed
all-reduce averages every gradient, the f64 scales included); rank 0 writes the
gradients (float.hex, exact) as JSON to argv[1]."""
import json
import os
import sys

import torch
import torch.distributed as dist
from torch.nn.parallel import DistributedDataParallel as DDP

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.ddp_common import batch, model, quant_grads  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    mode = os.environ.get("VSIQ_TEST_DEFERRED")
    m = model(launches=mode == "default")   # default: the reference flow's K7 + K4d
    if mode == "1":   # deferred qparam-gradient fold under DDP
        from vsiquantization_amd import enable_deferred_qparam_grads
        enable_deferred_qparam_grads(m)
    ddp = DDP(m, device_ids=[0])
    x = batch().chunk(world)[rank]
    ddp(x).square().sum().backward()
    grads = quant_grads(m)
    if rank == 0:
        out = {n: [v.hex() for v in g.double().reshape(-1).tolist()] for n, g in grads.items()}
        out["_dtypes"] = {n: str(g.dtype) for n, g in grads.items()}
        with open(sys.argv[1], "w") as f:
            json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
