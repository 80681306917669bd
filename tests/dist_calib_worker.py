"""Worker of tests/test_gpu_dist_calib.py: one rank of a batch-sharded calibration run
(launched by torch.distributed.run: 2 ranks, gloo, all ranks on cuda:0; or, with
VSIQ_DIST_BACKEND=nccl, ONE rank over RCCL -- RCCL does not put two ranks on one GPU,
and a 1-rank RCCL group still runs the real all_gather / all_reduce kernels and their
graph capture); argv: output path, configuration ("small" / "c5", tests/dist_calib_common.py).

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


def graph_replay(cfg, acts, shard):
    """A whole observe+quantize step of every layer (per call: K2p, the RCCL all_gather,
    the fold + fake-quant launch, and the STE backward) captured with GraphedStep: every
    replay == the eager step, bit for bit (the same inputs, so the observers' running
    min/max and qparams are fixed points after the first call)."""
    import numpy as np
    from tests.dist_calib_common import DEV
    from vsiquantization_amd.utils.graph import GraphedStep
    mgrs = managers(cfg)
    for qm in mgrs:
        qm.dist_group = dist.group.WORLD
        qm.is_quantize = True
    xs, gs = [], []
    for li, x in enumerate(acts[0]):
        gen = torch.Generator(device=DEV).manual_seed(70_000 + li)
        g = torch.randn(x.shape, device=DEV, generator=gen)
        xs.append(x.chunk(shard[1])[shard[0]].clone().requires_grad_(True))
        gs.append(g.chunk(shard[1])[shard[0]].contiguous())

    def step():
        ys = []
        for qm, x, g, (act, _) in zip(mgrs, xs, gs, cfg.layers):
            y = qm.quantize(x, act=act)
            y.backward(g)
            ys.append(y)
        return ys

    for x in xs:
        x.grad = None
    eager = [y.detach().clone() for y in step()]
    eager_g = [x.grad.clone() for x in xs]
    gstep = GraphedStep(step, grads_of=xs)
    ok = True
    for _ in range(3):
        ys = gstep()
        torch.cuda.synchronize()
        ok &= all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(ys, eager))
        ok &= all(torch.equal(x.grad.view(torch.int32), b.view(torch.int32)) for x, b in zip(xs, eager_g))
    from vsiquantization_amd import distributed as D
    ok &= D.capture_group() is not None   # the captured all_gathers ran on the capture-only twin
    return {"replays_equal_eager": bool(ok), "layers": len(xs),
            "y_sum": float(np.sum([float(y.double().sum()) for y in eager]))}


def main():
    out_path = sys.argv[1]
    cfg = Config(sys.argv[2] if len(sys.argv) > 2 else "small")
    backend = os.environ.get("VSIQ_DIST_BACKEND", "gloo")
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group(backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    acts = activations(cfg)
    res = {}
    for mode in ("per_call", "deferred"):
        mgrs = managers(cfg)
        for qm in mgrs:
            qm.dist_group = dist.group.WORLD
            qm.dist_defer = mode == "deferred"
        observe(cfg, mgrs, acts, shard=(rank, world))
        if mode == "deferred":
            # a read before the sync needs every rank's records: it raises on every
            # rank (no collective from one rank), and the sync still works afterwards
            try:
                float(mgrs[0].scale)
                res["deferred_read_raises"] = False
            except RuntimeError as e:
                res["deferred_read_raises"] = "sync_calibration" in str(e)
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
        if backend == "nccl":
            res["graph"] = graph_replay(cfg, acts, shard=(rank, world))
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
