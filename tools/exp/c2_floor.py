"""Is C2's forward (K3: per-channel observe + f64 qparams + fake quant + 1-bit mask,
vsiq_pc_observe_fq_f32) at the floor of its traffic mix on this box?  At C2's shape
(1024 x 9216 fp32, 8 buffers rotated past the 256 MB MALL), for every store gate in a
sweep (ticks of the 100 MHz wall clock; 0 = no gate), R launches back to back, event-timed:

  * K3 with the gate forced (VSIQ_TUNE_STORE_GATE),
  * the STE backward (vsiq_ste_bwd_f32: read g + the mask bits, write grad_x) with the
    same gate,
  * a plain gated copy of the same grid shape (c2_floor.hip: 9 float4 loads per lane, the
    gate, 9 stores; no reduction, no mask).

Prints us per launch for each and kernel / plain at each one's best gate.
usage: python tools/exp/c2_floor.py [reps]"""
import ctypes
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from vsiquantization_amd import _hip as H  # noqa: E402
from vsiquantization_amd.fakequant import qden  # noqa: E402

P = ctypes.c_void_p


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    so = os.path.join("/tmp", "c2_floor.so")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-o", so,
                    os.path.join(HERE, "c2_floor.hip")], check=True)
    dev = torch.device("cuda:0")
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    lib = H.lib()
    ex = ctypes.CDLL(so)
    ex.exp_copy_gated.argtypes = [P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint32, P]
    st = H.stream_of(dev)
    rows, rowlen, sl = 1024, 9216, 8
    g = torch.Generator(device=dev).manual_seed(0)
    xs = [torch.randn(rows, rowlen, device=dev, generator=g) * 0.05 for _ in range(sl)]
    ys = [torch.empty_like(xs[0]) for _ in range(sl)]
    mask = torch.empty(int(lib.vsiq_mask_words(H.c_i64(rows), H.c_i64(rowlen))), dtype=torch.int64, device=dev)
    run = torch.zeros(2, rows, device=dev)
    qp = torch.empty(2, rows, dtype=torch.float64, device=dev)
    qd = qden(False, 8, 1e-8)
    gs = [torch.randn(rows, rowlen, device=dev, generator=g) for _ in range(sl)]
    gxs = [torch.empty_like(xs[0]) for _ in range(sl)]

    def k3(i):
        j = i % sl
        return lib.vsiq_pc_observe_fq_f32(P(xs[j].data_ptr()), P(ys[j].data_ptr()), None, P(mask.data_ptr()),
                                          H.c_i64(rows), H.c_i64(rowlen), P(run[0].data_ptr()),
                                          P(run[1].data_ptr()), P(qp[0].data_ptr()), P(qp[1].data_ptr()), None, 0,
                                          0, 255, qd, 1e-8, st)

    def ste(i):
        j = i % sl
        return lib.vsiq_ste_bwd_f32(P(gs[j].data_ptr()), P(mask.data_ptr()), P(gxs[j].data_ptr()),
                                    H.c_i64(rows * rowlen), P(qp[0].data_ptr()), H.c_i64(rowlen), 0.0, st)

    def plain(gate):
        return lambda i: ex.exp_copy_gated(P(xs[i % sl].data_ptr()), P(ys[i % sl].data_ptr()), rows, rowlen, gate, st)

    def t(fn):
        for i in range(16):
            assert fn(i) == 0
        best = None
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(reps):
                fn(i)
            b.record()
            b.synchronize()
            us = a.elapsed_time(b) * 1e3 / reps
            best = us if best is None else min(best, us)
        return best

    alg = rows * rowlen * 8
    gates = [0] + list(range(440, 701, 13))
    res = []
    print(f"C2 shape {rows}x{rowlen}, {sl} buffers, {reps} launches per timing (min of 3)")
    print(" gate   K3 us  STE us  plain us")
    try:
        for gt in gates:
            H.set_tuning(H.TUNE_STORE_GATE, gt)
            a = t(k3)
            c = t(ste)
            b = t(plain(gt))
            res.append((gt, a, b, c))
            print(f"{gt:5d} {a:7.2f} {c:7.2f} {b:9.2f}", flush=True)
    finally:
        H.set_tuning(H.TUNE_STORE_GATE, -1)
    pa = min(res, key=lambda r: r[2])
    print(f"best plain copy {pa[2]:.2f} us at gate {pa[0]} = {alg / pa[2] / 1e3:.0f} GB/s ({alg / pa[2] / 8e6:.3f} of 8 TB/s)")
    for name, col in (("K3", 1), ("STE", 3)):
        ka = min(res, key=lambda r: r[col])
        print(f"best {name} {ka[col]:.2f} us at gate {ka[0]} = {alg / ka[col] / 1e3:.0f} GB/s "
              f"({alg / ka[col] / 8e6:.3f} of 8 TB/s); {pa[2] / ka[col]:.3f} of the plain copy's rate")


if __name__ == "__main__":
    main()
