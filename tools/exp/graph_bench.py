"""Host cost removed by HIP-graph capture: 27 small learnable fake-quant layers (fwd + bwd
through the public API), eager vs one torch.cuda.graph replay. Experiment only."""
import os, sys, time, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd as V  # noqa

dev = torch.device("cuda:0")
torch.manual_seed(0)
L = 27
qs = [V.UniformQuantizer(4, True) for _ in range(L)]
xs = [torch.randn(2, 32, 20, 20, device=dev, requires_grad=True) for _ in range(L)]
gs = [torch.randn(2, 32, 20, 20, device=dev) for _ in range(L)]
ss = [torch.nn.Parameter(torch.tensor(0.05, dtype=torch.float64, device=dev)) for _ in range(L)]


def step():
    ys = [q.quantize(x, s, 0, True, act="relu") for q, x, s in zip(qs, xs, ss)]
    torch.autograd.backward(ys, gs)


def wall(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


print(f"eager   27 layers fwd+bwd: {wall(step):8.1f} us/step", flush=True)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(3):
        step()
torch.cuda.current_stream().wait_stream(side)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
print(f"graph   27 layers fwd+bwd: {wall(g.replay):8.1f} us/step", flush=True)
