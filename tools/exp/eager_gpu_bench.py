"""The reference's own algorithm as eager PyTorch on the SAME MI355X (what running the
reference unchanged on PyTorch-ROCm would cost), against the HIP path, for C2 and C3.

Restated here op for op (the reference is not shipped to the GPU box and oracle/ is
test-only): quantizers/uniform.py:34-56 (x/s + zp, RoundStraightThrough, clamp,
(q - zp) * s, ScaleGradient on the learnable scale), observers/minmax.py:32-74
(x.min()/x.max() with .item(), float64 qparams on the host).  Per-channel (C2) has no
reference class: SURVEY §8c defines it as the reference classes looped over the
out-channels ("loop", 2 host syncs per channel); "vectorized" is the same arithmetic
as one batched torch expression (what a careful torch user would write).
Experiment only: prints one line per variant.
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import vsiquantization_amd as V  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)


class RoundSTE(torch.autograd.Function):          # uniform.py:258-271
    @staticmethod
    def forward(ctx, x):
        return torch.round(x)

    @staticmethod
    def backward(ctx, g):
        return g


class ScaleGradient(torch.autograd.Function):     # uniform.py:242-255
    @staticmethod
    def forward(ctx, x, scale):
        ctx.scale = scale
        return x

    @staticmethod
    def backward(ctx, g):
        return g * ctx.scale, None


def quantize(x, scale, zp, qmin, qmax):           # uniform.py:54-55, 95
    x_int = torch.clamp(RoundSTE.apply(x / scale + zp), qmin, qmax)
    return (x_int - zp) * scale


def observer_qparams(mn, mx, qmax=255, eps=1e-8):  # minmax.py:49-74, asymmetric
    s = (mx - mn) / (qmax + eps)
    return s, round(-mn / (s + eps))


def c2_loop(w, g):
    """Reference classes per out-channel: MinMaxObserver(False).forward(W[c]) then
    UniformQuantizer(8, False).quantize(W[c], s, zp, False); autograd backward."""
    wr = w.detach().requires_grad_(True)
    ys = []
    for c in range(w.shape[0]):
        row = wr[c]
        mn = min(0.0, row.min().item())           # minmax.py:42-47 (state starts at 0)
        mx = max(0.0, row.max().item())
        s, zp = observer_qparams(mn, mx)
        ys.append(quantize(row, s, zp, 0, 255))
    torch.stack(ys).backward(g)
    return wr.grad


def c2_vectorized(w, g):
    wr = w.detach().requires_grad_(True)
    x = wr.reshape(w.shape[0], -1)
    mn = torch.clamp(x.detach().amin(1), max=0.0).double()
    mx = torch.clamp(x.detach().amax(1), min=0.0).double()
    s = (mx - mn) / (255 + 1e-8)
    zp = torch.round(-mn / (s + 1e-8))
    y = quantize(x, s.float()[:, None], zp.float()[:, None], 0, 255)
    y.backward(g.reshape_as(y))
    return wr.grad


def c3_step(x, g, scale):
    """uniform.py:47-56, learnable symmetric int8 (zp = 0)."""
    xr = x.detach().requires_grad_(True)
    gs = (127 * x.numel()) ** -0.5                # uniform.py:58-71
    s = ScaleGradient.apply(scale, gs)
    y = quantize(xr, s, 0, -128, 127)
    y.backward(g)
    return xr.grad


def timed(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def hip_step(W, reps=50):
    for i in range(4):
        assert W.launch(i) == 0
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(reps):
        W.launch(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


W2 = bench.C2PerChannel(dev, 8, 0)
w, gw = W2.slots[0]["x"], W2.slots[0]["g"]
n2 = w.numel()
for name, fn, reps in (("loop", lambda: c2_loop(w, gw), 3), ("vectorized", lambda: c2_vectorized(w, gw), 20)):
    dt = timed(fn, reps)
    print(f"C2 eager torch {name:10s} {dt * 1e6:10.1f} us/step  {n2 / dt / 1e6:10.1f} Melem/s", flush=True)


def c2_api(w, g):
    """The same step through the public API (PerChannelMinMaxObserver + quantizer, autograd)."""
    wr = w.detach().requires_grad_(True)
    obs = V.PerChannelMinMaxObserver(False)
    y, _ = obs.observe_quantize(wr, V.PerChannelUniformQuantizer(8, False))
    y.backward(g)
    return wr.grad


dt = timed(lambda: c2_api(w, gw), 50)
print(f"C2 HIP via public API     {dt * 1e6:10.1f} us/step  {n2 / dt / 1e6:10.1f} Melem/s", flush=True)
dt = hip_step(W2, 200)
print(f"C2 HIP (bench.py path)    {dt * 1e6:10.1f} us/step  {n2 / dt / 1e6:10.1f} Melem/s", flush=True)
del W2, w, gw
torch.cuda.empty_cache()

W3 = bench.C3Lsq(dev, 2, 0)
x, g3 = W3.slots[0]["x"], W3.slots[0]["g"]
n3 = x.numel()
scale = torch.nn.Parameter(torch.tensor(0.03, dtype=torch.float64, device=dev))
dt = timed(lambda: c3_step(x, g3, scale), 10)
print(f"C3 eager torch learnable  {dt * 1e6:10.1f} us/step  {n3 / dt / 1e6:10.1f} Melem/s", flush=True)
q3 = V.UniformQuantizer(8, True)


def c3_api():
    xr = x.detach().requires_grad_(True)
    q3.quantize(xr, scale, 0, True).backward(g3)
    return xr.grad


dt = timed(c3_api, 20)
print(f"C3 HIP via public API     {dt * 1e6:10.1f} us/step  {n3 / dt / 1e6:10.1f} Melem/s", flush=True)
dt = hip_step(W3, 50)
print(f"C3 HIP (bench.py path)    {dt * 1e6:10.1f} us/step  {n3 / dt / 1e6:10.1f} Melem/s", flush=True)
