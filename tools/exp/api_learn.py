"""Host cost of the public API's learnable (LSQ) per-call path (experiment): one small
layer's activation fake quant with an f64 scale Parameter, forward + backward, through
UniformQuantizer.quantize and through QuantizationManager.quantize.  Prints us per step."""
import os, sys, time, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd as V  # noqa: E402

dev = torch.device("cuda:0")
shape = tuple(int(v) for v in os.environ.get("API_SHAPE", "8,16,20,20").split(","))
x = torch.randn(shape, device=dev).requires_grad_(True)
g = torch.randn_like(x)
q = V.UniformQuantizer(4, True)
s = torch.nn.Parameter(torch.tensor(0.05, dtype=torch.float64, device=dev))
qm = V.QuantizationManager("UniformQuantizer", "MinMaxObserver", 4, True, True)
qm.is_observer_qparam, qm.is_learning_scale, qm.is_quantize = True, False, False
qm.quantize(x.detach())
qm.is_learning_scale, qm.is_quantize = True, True
qm.init_scaling_factor_for_learning()
qm.make_learn_qparameter()


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


def quantizer_step():
    x.grad = None
    s.grad = None
    q.quantize(x, s, 0, True).backward(g)


def quantizer_relu_step():
    x.grad = None
    s.grad = None
    q.quantize(x, s, 0, True, act="relu").backward(g)


def manager_step():
    x.grad = None
    qm.scale.grad = None
    qm.quantize(x).backward(g)


def trivial():
    x.grad = None
    s.grad = None
    (x * s.float()).backward(g)


print(f"shape {shape}", flush=True)
for name, fn in (("UniformQuantizer fwd+bwd", quantizer_step), ("  + fused relu", quantizer_relu_step),
                 ("QuantizationManager fwd+bwd", manager_step), ("torch x*s fwd+bwd", trivial)):
    print(f"{name:30s} {t(fn):8.1f} us", flush=True)
