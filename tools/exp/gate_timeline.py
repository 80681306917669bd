"""Timeline of a K3-shaped one-round grid under different store gates (gate_timeline.hip).
Experiment only.  Times in us relative to the earliest workgroup start."""
import ctypes, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "gate_timeline.so"))
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
R, L = int(os.environ.get("ROWS", "1024")), 9216
xs = [torch.randn(R, L, device=dev) for _ in range(8)]
ys = [torch.empty(R, L, device=dev) for _ in range(8)]
rec = torch.zeros(R * 4, dtype=torch.int64, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = ctypes.c_void_p


def launch(i, gate):
    assert lib.exp_tl(P(xs[i % 8].data_ptr()), P(ys[i % 8].data_ptr()), ctypes.c_int64(R), ctypes.c_int64(L),
                      gate, P(rec.data_ptr()), st) == 0


gates = [int(g) for g in os.environ.get("GATES", "0 400 452 500 528 560 603 704").split()]
for rnd in range(2):
    for gate in gates:
        for i in range(8):
            launch(i, gate)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); s.record()
        for i in range(64):
            launch(i, gate)
        e.record(); torch.cuda.synchronize()
        us = s.elapsed_time(e) / 64 * 1e3
        spans, lines = [], []
        for i in range(6):    # a few single launches, timeline of each
            launch(i, gate); torch.cuda.synchronize()
            r = rec.view(R, 4).cpu().numpy().astype(np.int64)
            t0 = r[:, 0].min()
            q = lambda a, p: np.percentile((a - t0) / 100.0, p)
            spans.append((r[:, 3].max() - t0) / 100.0)
            lines.append(f"start p50/max {q(r[:,0],50):.2f}/{q(r[:,0],100):.2f}  land p10/50/90/99/max "
                         f"{q(r[:,1],10):.2f}/{q(r[:,1],50):.2f}/{q(r[:,1],90):.2f}/{q(r[:,1],99):.2f}/{q(r[:,1],100):.2f}"
                         f"  rel p50 {q(r[:,2],50):.2f}  end p50/max {q(r[:,3],50):.2f}/{q(r[:,3],100):.2f}"
                         f"  land-start(last-start wg) {(r[r[:,0].argmax(),1]-r[r[:,0].argmax(),0])/100:.2f}"
                         f"  max(land-start) {((r[:,1]-r[:,0]).max())/100:.2f}")
        print(f"gate {gate:4d}: events {us:6.2f} us; span med {np.median(spans):.2f}", flush=True)
        print("   " + lines[-1], flush=True)
