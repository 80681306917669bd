"""K6 / per-channel fake quant (LSQFakeQuantize per-channel, axis 1) at YOLOv8n activation
shapes, batch 256, and axis-0 weights. Experiment only: prints us and GB/s per launch.
Event-timed through the Python API: the first round of a shape includes the GPU's ramp
(round 5: K6 at 256x16x160x160 read 246-269 us in round 1, 206-208 from round 2; ROUNDS
defaults to 2), and small shapes are host-bound here (use rocprofv3 --kernel-trace for
their kernel time).  FLAT=1 adds K4 (per-tensor LSQ) on the same tensors."""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import vsiquantization_amd  # noqa
from vsiquantization_amd import fakequant as FQ

dev = torch.device("cuda:0")
from vsiquantization_amd import _hip as H  # noqa: E402
for kv in os.environ.get("TUNE", "").split():   # e.g. TUNE="11=0 10=0"
    k, v = kv.split("=")
    H.set_tuning(int(k), int(v))


def t(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(400):   # let the store-gate tuner settle this launch site first
        fn()
        if i % 16 == 15:
            torch.cuda.synchronize()
            if H.gate_tuning_pending() == 0:
                break
    torch.cuda.synchronize(); s.record()
    for _ in range(reps):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for shape, axis in (((256, 16, 160, 160), 1), ((256, 64, 40, 40), 1), ((256, 256, 10, 10), 1),
                    ((256, 128, 20, 20), 1), ((1024, 1024, 3, 3), 0)):
    if os.environ.get("SHAPE") and os.environ["SHAPE"] != "x".join(map(str, shape)):   # e.g. SHAPE=256x256x10x10
        continue
    nsets = max(1, -(-(768 << 20) // (12 * torch.Size(shape).numel())))   # rotate past the 256 MB MALL
    xs = [torch.randn(shape, device=dev) for _ in range(nsets)]
    gs = [torch.randn(shape, device=dev) for _ in range(nsets)]
    x = xs[0]
    C = shape[axis]
    s = torch.rand(C, dtype=torch.float64, device=dev) * 0.05 + 0.01
    z = torch.zeros(C, dtype=torch.float64, device=dev)
    n = x.numel()
    reps = max(10, min(200, (4 << 30) // (12 * n)))
    it = [0]

    def nxt():
        it[0] += 1
        return it[0] % nsets
    for rnd in range(int(os.environ.get("ROUNDS", "2"))):
        for alt in (os.environ.get("ALT", "").split(";") if os.environ.get("ALT") else [""]):
            for kv in alt.split():   # ALT="13=1;13=0": alternate knob settings, same process
                k, v = kv.split("=")
                H.set_tuning(int(k), int(v))
            fwd = t(lambda: FQ.per_channel_fake_quant(xs[nxt()], s, z, -128, 127, axis=axis), reps)
            bwd = t(lambda: (lambda i: FQ.pc_lsq_backward(gs[i], xs[i], s, z, -128, 127, 1e-4, True, axis))(nxt()),
                    reps)
            flat = ""
            if os.environ.get("FLAT", "0") == "1":   # K4 (per-tensor LSQ) on the same tensors: the floor
                s0 = torch.tensor(0.03, dtype=torch.float64, device=dev)
                fl = t(lambda: (lambda i: FQ.lsq_backward(gs[i], xs[i], s0, 0.0, -128, 127, 1e-4, False))(nxt()),
                       reps)
                flat = f"   K4 flat {fl:8.2f} us ({12 * n / fl / 1e3:5.0f} GB/s)"
            print(f"{str(shape):22s} axis {axis} {alt:8s} fwd {fwd:8.2f} us ({8 * n / fwd / 1e3:5.0f} GB/s)   "
                  f"bwd(K6) {bwd:8.2f} us ({12 * n / bwd / 1e3:5.0f} GB/s){flat}", flush=True)
