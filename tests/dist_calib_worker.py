"""Worker of tests/test_gpu_dist_calib.py: one rank of a batch-sharded calibration run
(launched by torch.distributed.run, 2 ranks, gloo, all ranks on cuda:0);
argv: output path, configuration ("small" / "c5", tests/dist_calib_common.py).

Every rank observes its half of every batch through QuantizationManager.quantize with
the managers' dist_group set -- per-call all-gather, or deferred K2p records + one
sync_calibration, and ("small") observe + quantize per call, whose y / gradients every
rank saves to argv[1].oq<rank>.npz -- and rank 0 writes the observer state as JSON to
argv[1]."""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.dist_calib_common import Config, activations, managers, observe, state  # noqa: E402
from vsiquantization_amd.distributed import sync_calibration  # noqa: E402


def main():
    out_path = sys.argv[1]
    cfg = Config(sys.argv[2] if len(sys.argv) > 2 else "small")
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    acts = activations(cfg)
    res = {}
    for mode in ("per_call", "deferred"):
        mgrs = managers(cfg)
        for qm in mgrs:
            qm.dist_group = dist.group.WORLD
            qm.dist_defer = mode == "deferred"
        observe(cfg, mgrs, acts, shard=(rank, world))
        if mode == "deferred":
            sync_calibration(torch.nn.ModuleList(mgrs))
            for qm in mgrs:
                qm.dist_defer = False
        res[mode] = state(mgrs)
    if cfg.name == "small":   # observe + quantize per call: gather + fold inside the fake quant
        import numpy as np
        from tests.dist_calib_common import observe_quantize
        mgrs = managers(cfg)
        for qm in mgrs:
            qm.dist_group = dist.group.WORLD
            qm.is_quantize = True
        np.savez(f"{out_path}.oq{rank}.npz", **observe_quantize(cfg, mgrs, acts, shard=(rank, world)))
        res["observe_quantize"] = state(mgrs)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
