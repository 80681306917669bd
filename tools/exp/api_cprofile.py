"""cProfile of the C2 public-API step (host Python cost by function). Experiment only."""
import cProfile, os, pstats, sys, time, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd as V  # noqa
from vsiquantization_amd import _hip as H
dev = torch.device("cuda:0")
w = torch.randn(1024, 1024, 3, 3, device=dev) * 0.05
g = torch.randn_like(w)
q = V.PerChannelUniformQuantizer(8, False)


def step():
    wr = w.detach().requires_grad_(True)
    obs = V.PerChannelMinMaxObserver(False)
    y, _ = obs.observe_quantize(wr, q)
    y.backward(g)


for _ in range(50):
    step()
torch.cuda.synchronize()
N = 2000
t = time.perf_counter()
for _ in range(N):
    step()
torch.cuda.synchronize()
print(f"step {(time.perf_counter() - t) / N * 1e6:.1f} us", flush=True)
for name, fn in (("current_stream", lambda: torch.cuda.current_stream(dev)), ("stream_of", lambda: H.stream_of(dev)),
                 ("ptr", lambda: H.ptr(w)), ("empty_like", lambda: torch.empty_like(w)),
                 ("zeros1024", lambda: torch.zeros(1024, device=dev)), ("mask_buffer", lambda: H.mask_buffer(1024, 9216, dev)),
                 ("mask_words", lambda: H.lib().vsiq_mask_words(1024, 9216))):
    t = time.perf_counter()
    for _ in range(N):
        fn()
    torch.cuda.synchronize()
    print(f"{name:16s} {(time.perf_counter() - t) / N * 1e6:.2f} us", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    step()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
