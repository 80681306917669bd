"""Does an event recorded between two kernels on one stream take its timestamp after the
first kernel has finished?  Kernel A (a ~100 us streaming pass), event a, kernel B (a short
K1 fake quant), event b: elapsed(a, b) against B timed alone after a sync, for HIP events
with hipEventDisableSystemFence (bench.HipEvent, the tuner's) and torch's default events.
usage: python tools/exp/event_order.py"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vsiquantization_amd import fakequant as FQ  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    big = torch.randn(1 << 27, device=dev)          # 512 MB: A reads + writes it (~150 us)
    small = torch.randn(1 << 20, device=dev)        # B: K1 on 1M elements (~4 us)
    out = torch.empty_like(small)

    def kb():
        FQ.fake_quant(small, 0.05, 0.0, -128, 127)

    for kind, mk in (("hip DisableSystemFence", bench.HipEvent), ("torch default", lambda: torch.cuda.Event(enable_timing=True))):
        alone, after = [], []
        for _ in range(20):
            torch.cuda.synchronize()
            a, b = mk(), mk()
            a.record()
            kb()
            b.record()
            torch.cuda.synchronize()
            alone.append(a.elapsed_time(b) * 1e3)
            a, b, c = mk(), mk(), mk()
            c.record()
            big.mul_(1.0)                             # A
            a.record()
            kb()
            b.record()
            torch.cuda.synchronize()
            after.append(a.elapsed_time(b) * 1e3)
            ta = c.elapsed_time(a) * 1e3
        print(f"{kind:24s}: B alone {statistics.median(alone):7.2f} us, B after A {statistics.median(after):7.2f} us "
              f"(A measured {ta:7.2f} us)", flush=True)
    _ = out


if __name__ == "__main__":
    main()
