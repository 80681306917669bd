"""Batched activation quant (bench.ActQuant: per layer K2 observe, then K1 fake quant of
the same tensor, fused ReLU, 12 B/elem algorithmic) at the per-GPU batch of N = 1 / 4 / 8
ranks (1024 / 256 / 128 images), with K2's loads nontemporal (default) or cached
(VSIQ_TUNE_OBS_TEMPORAL_MB): does K1's second read of a layer hit the 256 MB Infinity
Cache once the layer fits it?  Event-timed steps (27 layers), median of 5 x R steps.
usage: python tools/exp/act_mall.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vsiquantization_amd import _hip as H  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    for batch in (128, 256, 1024):
        W = bench.ActQuant(dev, 1, 0, total_batch=batch)
        biggest = max(t["x"].numel() for t in W.L) * 4 / 2 ** 20
        row = []
        for mb in (0, 64, 128, 192, 256):
            H.set_tuning(H.TUNE_OBS_TEMPORAL_MB, mb)
            reps = max(4, 2048 // batch)
            for i in range(3):
                assert W.launch(i) == 0
            ts = []
            for _ in range(5):
                e0, e1 = bench.HipEvent(), bench.HipEvent()
                torch.cuda.synchronize()
                e0.record()
                for i in range(reps):
                    W.launch(i)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / reps)
            us = sorted(ts)[2]
            row.append(f"temporal<{mb}MB: {us:9.1f} us {12 * W.n / us / 1e3:6.0f} GB/s(alg)")
        H.set_tuning(H.TUNE_OBS_TEMPORAL_MB, 0)
        assert W.check()
        print(f"batch {batch:5d} ({W.n / 1e6:.0f}M elem, largest layer {biggest:.0f} MB): " + " | ".join(row),
              flush=True)
        del W
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
