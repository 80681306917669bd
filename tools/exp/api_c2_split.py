"""Where the public-API C2 step's time goes (experiment): forward and backward timed
apart (each bracketed by a device sync), the same for torch's own x * 1.0, and the step
with the store gate off.  1024x1024x3x3 weights, 4 in rotation, on a side stream like
bench.py.  Prints us per step (median of 7 runs of 40)."""
import os, sys, time, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

dev = torch.device("cuda:0")
if os.environ.get("SIDE_STREAM", "1") == "1":
    torch.cuda.set_stream(torch.cuda.Stream(dev))
import vsiquantization_amd as V  # noqa: E402
from vsiquantization_amd import _hip as H  # noqa: E402

xs = [(torch.randn(1024, 1024, 3, 3, device=dev) * 0.05).requires_grad_(True) for _ in range(4)]
g = torch.randn_like(xs[0])
obs, q = V.PerChannelMinMaxObserver(False), V.PerChannelUniformQuantizer(8, False)


def med(fn, n=40, reps=7):
    for i in range(30):
        fn(i)
    res = []
    for _ in range(reps):
        acc = 0.0
        for i in range(n):
            acc += fn(i)
        res.append(acc / n * 1e6)
    return sorted(res)[reps // 2]


def timed(f):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    f()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def api_step(i):
    x = xs[i % 4]
    x.grad = None
    return timed(lambda: obs.observe_quantize(x, q)[0].backward(g))


def torch_step(i):
    x = xs[i % 4]
    x.grad = None
    return timed(lambda: (x * 1.0).backward(g))


def api_split(which):
    def f(i):
        x = xs[i % 4]
        x.grad = None
        box = []
        tf = timed(lambda: box.append(obs.observe_quantize(x, q)[0]))
        tb = timed(lambda: box[0].backward(g))
        return tf if which == "f" else tb
    return f


def torch_split(which):
    def f(i):
        x = xs[i % 4]
        x.grad = None
        box = []
        tf = timed(lambda: box.append(x * 1.0))
        tb = timed(lambda: box[0].backward(g))
        return tf if which == "f" else tb
    return f


def api_step_nosync(i):   # like bench.py: no sync between steps
    x = xs[i % 4]
    x.grad = None
    t0 = time.perf_counter()
    obs.observe_quantize(x, q)[0].backward(g)
    return time.perf_counter() - t0


def torch_step_nosync(i):
    x = xs[i % 4]
    x.grad = None
    t0 = time.perf_counter()
    (x * 1.0).backward(g)
    return time.perf_counter() - t0


rows = [("api step (synced)", api_step), ("torch x*1 step (synced)", torch_step),
        ("api fwd alone", api_split("f")), ("api bwd alone", api_split("b")),
        ("torch fwd alone", torch_split("f")), ("torch bwd alone", torch_split("b")),
        ("api step host-only (no sync)", api_step_nosync), ("torch step host-only (no sync)", torch_step_nosync)]
if os.environ.get("SPLIT", "1") == "1":
    for name, fn in rows:
        print(f"{name:32s} {med(fn):8.1f} us", flush=True)
    H.set_tuning(12, 0)   # gate autotune off
    H.set_tuning(11, 0)   # gate off
    print(f"{'api step, store gate off':32s} {med(api_step):8.1f} us", flush=True)
    print(f"{'api bwd alone, store gate off':32s} {med(api_split('b')):8.1f} us", flush=True)

# interleaved: tuned gate / gate off / torch, 15 reps of 40 synced + unsynced steps
if os.environ.get("INTERLEAVE", "1") == "1":
    def run(fn, gate, n=40):
        H.set_tuning(11, gate)
        for i in range(5):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            fn(i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e6

    def api(i):
        xs[i % 4].grad = None
        obs.observe_quantize(xs[i % 4], q)[0].backward(g)

    def tor(i):
        xs[i % 4].grad = None
        (xs[i % 4] * 1.0).backward(g)

    H.set_tuning(12, 1)
    res = {"tuned gate": [], "gate off": [], "torch": []}
    for r in range(15):
        res["tuned gate"].append(run(api, -1))
        res["gate off"].append(run(api, 0))
        res["torch"].append(run(tor, -1))
    for k, v in res.items():
        v.sort()
        print(f"interleaved {k:12s} median {v[7]:7.1f} us  min {v[0]:7.1f}  max {v[-1]:7.1f}", flush=True)
    print(H.gate_report() if hasattr(H, "gate_report") else "", flush=True)
