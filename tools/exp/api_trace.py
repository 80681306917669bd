"""The public-API C2 step in a loop (no sync between steps), for a rocprofv3 kernel trace
(experiment): prints the host time per step; the trace shows the kernels' durations
and the gaps between them.  MODE=torch runs torch's own (x * 1.0).backward(g) instead."""
import os, sys, time, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

dev = torch.device("cuda:0")
torch.cuda.set_stream(torch.cuda.Stream(dev))
import vsiquantization_amd as V  # noqa: E402

xs = [(torch.randn(1024, 1024, 3, 3, device=dev) * 0.05).requires_grad_(True) for _ in range(4)]
g = torch.randn_like(xs[0])
obs, q = V.PerChannelMinMaxObserver(False), V.PerChannelUniformQuantizer(8, False)
mode = os.environ.get("MODE", "api")
for kv in filter(None, os.environ.get("TUNE", "").split(",")):   # e.g. TUNE=12=0 (gate autotune off)
    k, v = kv.split("=")
    V._hip.set_tuning(int(k), int(v))


def step(i):
    x = xs[i % 4]
    x.grad = None
    if mode == "torch":
        (x * 1.0).backward(g)
    else:
        obs.observe_quantize(x, q)[0].backward(g)


for i in range(100):
    step(i)
for r in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(200):
        step(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{mode}: {(t2 - t0) / 200 * 1e6:.1f} us/step, host enqueue {(t1 - t0) / 200 * 1e6:.1f} us/step",
          flush=True)
