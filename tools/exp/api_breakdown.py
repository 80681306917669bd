"""Host cost breakdown of the C2 step through the public API (experiment): forward only,
forward + backward, a trivial torch autograd op fwd + bwd (the engine's own cost), and
a bare kernel-free torch op, all on one 1024x1024x3x3 weight.  Prints us per step."""
import os, sys, time, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd as V  # noqa: E402

dev = torch.device("cuda:0")
x = (torch.randn(1024, 1024, 3, 3, device=dev) * 0.05).requires_grad_(True)
g = torch.randn_like(x)
obs, q = V.PerChannelMinMaxObserver(False), V.PerChannelUniformQuantizer(8, False)


def t(fn, n=300):
    for _ in range(30):
        fn()
    res = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n // 5):
            fn()
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) / (n // 5) * 1e6)
    return sorted(res)[2]


def fwd():
    with torch.no_grad():
        obs.observe_quantize(x, q)


def fwd_graph():
    obs.observe_quantize(x, q)


def step():
    x.grad = None
    y, _ = obs.observe_quantize(x, q)
    y.backward(g)


def trivial():
    x.grad = None
    (x * 1.0).backward(g)


def empty():
    torch.empty_like(x)


from vsiquantization_amd import _hip as H  # noqa: E402
from vsiquantization_amd.fakequant import qden  # noqa: E402
ext = H.torch_ext()
mn, mx = obs._state(x)
qd = qden(False, 8, 1e-8)


def ext_fwd():
    ext.pc_observe_fq(x, mn, mx, False, 0, 255, qd, 1e-8, False)


def ext_step():
    x.grad = None
    y = ext.pc_observe_fq(x, mn, mx, False, 0, 255, qd, 1e-8, False)[0]
    y.backward(g)


def py_wrapper_only():
    H.require_device_f32(x)
    obs._state(x)
    H.torch_ext_enabled()
    qden(False, 8, 1e-8)


for name, fn in (("fwd (no grad)", fwd), ("fwd (autograd node)", fwd_graph), ("fwd + bwd", step),
                 ("torch x*1 fwd + bwd", trivial), ("torch.empty_like", empty),
                 ("ext fwd (direct)", ext_fwd), ("ext fwd + bwd (direct)", ext_step),
                 ("python wrapper only", py_wrapper_only)):
    print(f"{name:22s} {t(fn):8.1f} us", flush=True)
