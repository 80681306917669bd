"""C2 launch-rate probe: is the event-timed K3/STE figure host-bound or GPU-bound?
(a) host enqueue time per K3 launch (ctypes + gate select + hipLaunchKernel, no sync);
(b) event span per launch for runs of N back-to-back K3 launches (8 slots rotated),
    started right after a sync (the bench's situation) and behind a 2 ms GPU sleep
    (host already ahead: the GPU never waits for a launch)."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "..", ".."))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    W = bench.C2PerChannel(dev, 8, 0)
    for i in range(300):
        W.launch(i)
    torch.cuda.synchronize()
    f = W.f_fwd
    args = [s["fwd"] for s in W.slots]
    # (a) host enqueue rate
    for n in (64, 512):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            f(*args[i % 8])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"host enqueue {n} K3: {1e6 * (t1 - t0) / n:.2f} us/launch; GPU done {1e6 * (t2 - t0) / n:.2f} us/launch")
    # (b) event spans
    for sleep in (False, True):
        for n in (1, 2, 8, 64, 256):
            reps = []
            for r in range(5):
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if sleep:
                    torch.cuda._sleep(2_000_000)
                a.record()
                for i in range(n):
                    f(*args[i % 8])
                b.record()
                torch.cuda.synchronize()
                reps.append(1e3 * a.elapsed_time(b) / n)
            reps.sort()
            print(f"{'behind sleep' if sleep else 'after sync  '} N={n:4d}: {reps[2]:.2f} us/launch (min {reps[0]:.2f})")


if __name__ == "__main__":
    main()
