"""Worker of tests/test_gpu_dist_calib.py: one rank of a batch-sharded calibration run
(launched by torch.distributed.run, 2 ranks, gloo, all ranks on cuda:0).

Every rank builds the same 3-layer ConvBnReLU model (seeded), takes its half of every
calibration batch, runs calibrate_qat_model with the activation observers' dist_group
set (per-call all-reduce, or deferred records + one sync_calibration), and rank 0
writes the observer state as JSON to argv[1]."""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.dist_calib_common import DEV, loader, model, state  # noqa: E402
from vsiquantization_amd.utils.quantize_manager import calibrate_qat_model, data_calib  # noqa: E402


def main():
    out_path = sys.argv[1]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    res = {}
    for mode in ("per_call", "deferred"):
        m = model()
        for layer in m:
            layer.activation_quantizer.dist_group = dist.group.WORLD
        shard = [(imgs.chunk(world)[rank], t) for imgs, t in loader()]
        calibrate_qat_model(m, shard, data_calib, DEV, defer_observers=(mode == "deferred"))
        res[mode] = state(m)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
