"""K3 (C2 forward) with and without the 1-bit straight-through mask: per-launch time
(256 back-to-back launches over 8 slots behind a GPU sleep, fence-free HIP events) ->
does the mask's 8-byte-per-lane store pattern cost more than its 1.6 % of the bytes?
Run under `rocprofv3 --pmc WRITE_SIZE` to compare the write counters of the two."""
import sys

import torch

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "..", ".."))
import bench  # noqa: E402


def timed(f, args, n=256, reps=5):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        a, b = bench.HipEvent(), bench.HipEvent()
        torch.cuda._sleep(2_000_000)
        a.record()
        for i in range(n):
            assert f(*args[i % len(args)]) == 0
        b.record()
        torch.cuda.synchronize()
        out.append(1e3 * a.elapsed_time(b) / n)
    return sorted(out)[reps // 2]


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    W = bench.C2PerChannel(dev, 8, 0)
    with_mask = [s["fwd"] for s in W.slots]
    no_mask = [s["fwd"][:3] + (None,) + s["fwd"][4:] for s in W.slots]
    for args in (with_mask, no_mask):   # settle both gate sites (same site: same kernel? no)
        for i in range(2000):
            W.f_fwd(*args[i % 8])
            if i % 64 == 63:
                torch.cuda.synchronize()
    torch.cuda.synchronize()
    for r in range(3):
        tm, tn = timed(W.f_fwd, with_mask), timed(W.f_fwd, no_mask)
        alg_m, alg_n = W.kernels["pc_observe_fq_fwd"], 8 * W.n
        print(f"with mask {tm:.2f} us ({alg_m / tm / 1e3:.0f} GB/s)   no mask {tn:.2f} us ({alg_n / tn / 1e3:.0f} GB/s)"
              f"   mask cost {100 * (tm / tn - 1):.2f} % for {100 * (alg_m / alg_n - 1):.2f} % more bytes")
    from vsiquantization_amd import _hip as H
    print(H.gate_report())


if __name__ == "__main__":
    main()
