"""Host cost of the public-API per-channel step, piece by piece, on a SMALL weight (GPU
time per launch ~3 us, so the loop is host-bound and the figures are host costs).
Experiment only."""
import os, sys, time, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd as V  # noqa
from vsiquantization_amd import _hip as H
dev = torch.device("cuda:0")
shape = tuple(int(v) for v in os.environ.get("SHAPE", "64x16x3x3").split("x"))
w = (torch.randn(shape, device=dev) * 0.05).requires_grad_(True)
g = torch.randn_like(w)
obs, q = V.PerChannelMinMaxObserver(False), V.PerChannelUniformQuantizer(8, False)
ext = H.torch_ext()
mn, mx = obs._state(w)
N = 3000


def timeit(name, fn):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(N):
        fn()
    torch.cuda.synchronize()
    print(f"{name:34s} {(time.perf_counter() - t) / N * 1e6:7.2f} us", flush=True)


def step():
    w.grad = None
    y, _ = obs.observe_quantize(w, q)
    y.backward(g)


def fwd():
    obs.observe_quantize(w, q)


def fwd_ext():
    ext.pc_observe_fq(w, mn, mx, False, 0, 255, 255 + 1e-8, 1e-8, False)


def step_ext():
    w.grad = None
    y = ext.pc_observe_fq(w, mn, mx, False, 0, 255, 255 + 1e-8, 1e-8, False)[0]
    torch.autograd.backward([y], [g])


def step_ext_engine():
    w.grad = None
    y = ext.pc_observe_fq(w, mn, mx, False, 0, 255, 255 + 1e-8, 1e-8, False)[0]
    torch._C._EngineBase.run_backward  # noqa
    torch.autograd.graph.Node  # noqa
    torch.autograd.backward(y, g)


C = shape[0]
rowlen = w.numel() // C
y0, gx0 = torch.empty_like(w), torch.empty_like(w)
sc, zp = torch.empty(C, dtype=torch.float64, device=dev), torch.empty(C, dtype=torch.float64, device=dev)
mask = H.mask_buffer(C, rowlen, dev)
st = H.stream_of(dev)
lib = H.lib()
fa = (H.ptr(w), H.ptr(y0), None, H.ptr(mask), H.c_i64(C), H.c_i64(rowlen), H.ptr(mn), H.ptr(mx), H.ptr(sc),
      H.ptr(zp), None, 0, 0, 255, 255 + 1e-8, 1e-8, st)
ba = (H.ptr(g), H.ptr(mask), H.ptr(gx0), H.c_i64(w.numel()), H.ptr(sc), H.c_i64(rowlen), 0.0, st)
timeit("C ABI fwd+bwd launches (ctypes)", lambda: (lib.vsiq_pc_observe_fq_f32(*fa), lib.vsiq_ste_bwd_f32(*ba)))
timeit("C ABI fwd launch (ctypes)", lambda: lib.vsiq_pc_observe_fq_f32(*fa))
timeit("ext fwd (pybind + C++ node)", fwd_ext)
timeit("ext fwd + autograd.backward", step_ext)
timeit("public fwd (observe_quantize)", fwd)
timeit("public step (fwd + y.backward)", step)
timeit("torch.empty_like", lambda: torch.empty_like(w))
with torch.no_grad():
    timeit("public fwd, no grad", fwd)
