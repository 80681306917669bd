"""Worker of tests/test_gpu_bench_capture.py (one rank under torch.distributed.run,
RCCL): bench.ActQuant with the per-call exchange forced on (per layer K2 records, the
RCCL all_gather, the K1r fold + fake quant), launched directly and then through
bench.capture_groups' HIP graphs (the collective inside the capture) -> outputs and
qparams bit for bit; then bench.measure over it.  Prints one JSON line."""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    import vsiquantization_amd  # noqa: F401
    W = bench.ActQuant(dev, 1, 0, total_batch=8, exchange=True)
    for i in range(3):
        assert W.launch(i) == 0
    torch.cuda.synchronize()
    ref = [(t["y"].clone(), t["qp"].clone(), t["rmm"].clone()) for t in W.L]
    for t in W.L:
        t["y"].fill_(float("nan"))
    caps = bench.capture_groups(W, [(0, 2)], len(W.kernels))
    assert caps is not None, "capture failed"
    for _ in range(2):
        for g in caps[0]:
            g.replay()
    torch.cuda.synchronize()
    same = all(torch.equal(t["y"].view(torch.int32), y.view(torch.int32)) and torch.equal(t["qp"], qp)
               and torch.equal(t["rmm"], rmm) for t, (y, qp, rmm) in zip(W.L, ref))
    r = bench.measure(W, 4, 2, 1)
    from vsiquantization_amd import distributed as D
    twin = D.capture_group()
    # the world still runs eager collectives after the captures (its stream never joined one)
    t = torch.ones(1, device=dev)
    dist.all_reduce(t)
    print(json.dumps({"graph_equals_direct": bool(same), "launch": r["launch"], "self_check": r["self_check"],
                      "alt": r.get("alt_launch", {}).get("launch"), "frac": r["roofline"]["frac"],
                      "capture_twin": twin is not None and twin is not dist.group.WORLD,
                      "world_after": float(t)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
