"""Host cost of the public-API C2 step, split by layer (experiment).  A 64x4x3x3 weight
keeps every kernel at its launch floor, so the times are host-bound: the Python wrapper
(observe_quantize), the pybind call into the C++ autograd node alone, the engine's
backward, and torch's own trivial op for comparison.  Prints us per step."""
import os, sys, time, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd as V  # noqa: E402
from vsiquantization_amd import _hip as H  # noqa: E402
from vsiquantization_amd.fakequant import qden  # noqa: E402

dev = torch.device("cuda:0")
shape = tuple(int(v) for v in os.environ.get("API_SHAPE", "64,4,3,3").split(","))
x = (torch.randn(shape, device=dev) * 0.05).requires_grad_(True)
g = torch.randn_like(x)
obs, q = V.PerChannelMinMaxObserver(False), V.PerChannelUniformQuantizer(8, False)
ext = H.torch_ext()
mn, mx = obs._state(x)
qd = qden(False, 8, obs.eps)


def t(fn, n=1000):
    for _ in range(50):
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


def api_fwd_nograd():
    with torch.no_grad():
        obs.observe_quantize(x, q)


def api_fwd():
    obs.observe_quantize(x, q)


def api_step():
    x.grad = None
    y, _ = obs.observe_quantize(x, q)
    y.backward(g)


def ext_fwd():
    ext.pc_observe_fq(x, mn, mx, False, 0, 255, qd, obs.eps, False)


def ext_step():
    x.grad = None
    y = ext.pc_observe_fq(x, mn, mx, False, 0, 255, qd, obs.eps, False)[0]
    y.backward(g)


def ext_step_autograd_grad():
    torch.autograd.grad(ext.pc_observe_fq(x, mn, mx, False, 0, 255, qd, obs.eps, False)[0], x, g)


KEEP = []


def ext_step_keep():
    x.grad = None
    out = ext.pc_observe_fq(x, mn, mx, False, 0, 255, qd, obs.eps, False)
    KEEP[:] = out[1:]
    out[0].backward(g)


def api_step_drop():
    x.grad = None
    y, _ = obs.observe_quantize(x, q)
    obs.scale = obs.zero_point = None
    y.backward(g)


def api_step_sync_free():
    x.grad = None
    xx = H.require_device_f32(x)
    y = ext.pc_observe_fq(xx, mn, mx, bool(obs.symmetric), int(q.qmin), int(q.qmax), qd, float(obs.eps),
                          False)[0]
    y.backward(g)


def trivial():
    x.grad = None
    (x * 1.0).backward(g)


def trivial_fwd():
    x * 1.0


print(f"shape {shape}", flush=True)
for name, fn in (("api fwd (no grad)", api_fwd_nograd), ("api fwd (node)", api_fwd), ("api fwd + bwd", api_step),
                 ("ext fwd (node)", ext_fwd), ("ext fwd + bwd", ext_step),
                 ("ext fwd + autograd.grad", ext_step_autograd_grad),
                 ("ext fwd + bwd, outs kept", ext_step_keep), ("api fwd + bwd, qparams dropped", api_step_drop),
                 ("ext + api arg prep", api_step_sync_free), ("api fwd + bwd (again)", api_step),
                 ("torch x*1 fwd", trivial_fwd), ("torch x*1 fwd + bwd", trivial)):
    print(f"{name:26s} {t(fn):8.1f} us", flush=True)
