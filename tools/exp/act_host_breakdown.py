"""Per-step host-time breakdown of the batched activation quant at N ranks (run under
torchrun; VSIQ_BENCH_BACKEND=gloo rehearses N=2 on one GPU).  Times, per step of the
27 layers, the host side of each operation of the per-call exchange:

  round 3 (K1r): K2 launch | all_gather_into_tensor | fold + fake-quant launch
  round 2:       K2 launch | all_gather             | finalize launch | K1 launch

and the step's wall time (synchronized).  Usage:
  VSIQ_BENCH_BACKEND=gloo torchrun --nproc-per-node 2 tools/exp/act_host_breakdown.py
"""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402


def main():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    backend = os.environ.get("VSIQ_BENCH_BACKEND", "nccl")
    dev = torch.device("cuda", 0 if backend != "nccl" else int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    dist.init_process_group(backend)
    W = bench.ActQuant(dev, world, rank, total_batch=int(os.environ.get("ACT_BATCH", "256")))
    lib = W.H.lib()
    for t in W.L:   # round-2 sequence for comparison: finalize launch + K1 launch
        P = t["rfq"]
        t["fin"] = (P[6], world, P[8], P[9], P[10], 1, P[12], 1e-8, P[16])
    pc = time.perf_counter

    def step(new, acc):
        for t in W.L:
            t0 = pc()
            lib.vsiq_act_observe_f32(*t["obs"])
            t1 = pc()
            dist.all_gather_into_tensor(t["gat"], t["st"])
            t2 = pc()
            if new:
                lib.vsiq_act_fq_fwd_ranks_f32(*t["rfq"])
                t3 = t4 = pc()
            else:
                lib.vsiq_observe_finalize_ranks(*t["fin"])
                t3 = pc()
                lib.vsiq_act_fq_fwd_f32(*t["fq"])
                t4 = pc()
            acc[0] += t1 - t0
            acc[1] += t2 - t1
            acc[2] += t3 - t2
            acc[3] += t4 - t3

    for new in (False, True, False, True):
        for _ in range(3):
            step(new, [0.0] * 4)
        torch.cuda.synchronize()
        dist.barrier()
        acc, steps = [0.0] * 4, 20
        t0 = pc()
        for _ in range(steps):
            step(new, acc)
        torch.cuda.synchronize()
        wall = (pc() - t0) / steps
        if rank == 0:
            names = ("K2 launch", "all_gather", "fold+fq launch" if new else "finalize launch", "-" if new else "K1 launch")
            parts = ", ".join(f"{n} {1e6 * a / steps:.0f} us" for n, a in zip(names, acc) if n != "-")
            print(f"{'round 3 K1r' if new else 'round 2    '}: {len(W.L)} layers, host per step: {parts}; "
                  f"host ops per step {len(W.L) * (3 if new else 4)}; wall {1e3 * wall:.2f} ms/step", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
