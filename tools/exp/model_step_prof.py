"""cProfile of the end-to-end QAT training step (tools/exp/model_step.py's 'ours' form,
per-call and deferred + multi-tensor) at a host-bound batch: where the Python time of the
fused layers goes (experiment).  Prints the top functions by own time per step."""
import cProfile
import io
import os
import pstats
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "exp"))
import model_step as M  # noqa: E402

STEPS = 20


def profile(name, m, x):
    step = M.step_fn(m, x)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(STEPS):
        step()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    print(f"== {name}: {st.total_tt / STEPS * 1e3:.2f} ms of profiled Python per step", flush=True)
    st.sort_stats("tottime").print_stats(22)
    print("\n".join(l for l in s.getvalue().splitlines() if l.strip())[:6000], flush=True)


def main():
    x = (torch.randint(0, 256, (M.BATCH, 3, 320, 320), generator=torch.Generator().manual_seed(9),
                       dtype=torch.uint8).float() / 255).to(M.dev)
    profile("ours (per call)", M.ours(M.chain()), x)
    plus = M.ours(M.chain())
    M.enable_multi_tensor_weights(plus)
    M.enable_deferred_qparam_grads(plus)
    profile("ours + K7 weights + K4d deferred", plus, x)


if __name__ == "__main__":
    main()
