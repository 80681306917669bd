"""C2 forward with the uint8 integer codes emitted as well (8 B/elem, plus 1 B/elem
when the codes are written -- report both).  K3 with mask only (bench.py's C2) vs mask +
codes, event-timed over 8 rotating slots.  Experiment only."""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa
from vsiquantization_amd import _hip as H
dev = torch.device("cuda:0")
W = bench.C2PerChannel(dev, 8, 0)
codes = [torch.empty(W.shape, dtype=torch.uint8, device=dev) for _ in W.slots]
n = W.n
mbytes = 8 * int(H.lib().vsiq_mask_words(W.shape[0], W.rowlen))


def t(fn, reps=400):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(16):
        fn(i)
    torch.cuda.synchronize(); s.record()
    for i in range(reps):
        fn(i)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def fwd_codes(i):
    a = list(W.slots[i % 8]["fwd"])
    a[2] = H.ptr(codes[i % 8])
    return W.f_fwd(*a)


for rnd in range(2):
    m = t(lambda i: W.f_fwd(*W.slots[i % 8]["fwd"]))
    c = t(fwd_codes)
    print(f"K3 mask only   {m:6.2f} us  {(8 * n + mbytes) / m / 1e3:6.0f} GB/s  ({(8 * n + mbytes) / 1e6:.1f} MB)")
    print(f"K3 mask+codes  {c:6.2f} us  {(9 * n + mbytes) / c / 1e3:6.0f} GB/s  ({(9 * n + mbytes) / 1e6:.1f} MB)", flush=True)
