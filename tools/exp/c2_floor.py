"""Is C2's forward (K3: per-channel observe + f64 qparams + fake quant + 1-bit mask,
vsiq_pc_observe_fq_f32) at the floor of its traffic mix on this box?  At C2's shape
(1024 x 9216 fp32, 8 buffers rotated past the 256 MB MALL), for every store gate in a
sweep (ticks of the 100 MHz wall clock; 0 = no gate), R launches back to back, event-timed:

  * K3 with the gate forced (VSIQ_TUNE_STORE_GATE),
  * the STE backward (vsiq_ste_bwd_f32: read g + the mask bits, write grad_x) with the
    same gate,
  * the learnable per-channel forward (vsiq_pcm_fq_fwd_f32: given f64 scale / zp per row,
    zp rounded, no observer; bench.py's pc_learn_fwd leg) with the same gate, without
    and with the 1-bit mask, and its backward K6 (vsiq_pcm_lsq_bwd_f32, zp learned: read g, x,
    write grad_x, 12 B/elem; bench.py's pc_learn_bwd_k6 leg),
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

    sc = torch.rand(rows, dtype=torch.float64, device=dev, generator=g) * 0.002 + 0.0005
    zp = torch.rand(rows, dtype=torch.float64, device=dev, generator=g) * 8 - 4

    def pcm(with_mask):
        mp = P(mask.data_ptr()) if with_mask else None
        return lambda i: lib.vsiq_pcm_fq_fwd_f32(P(xs[i % sl].data_ptr()), P(ys[i % sl].data_ptr()), None, mp,
                                                 H.c_i64(rows), H.c_i64(rowlen), H.c_i64(rows), P(sc.data_ptr()),
                                                 P(zp.data_ptr()), 1, -128, 127, st)

    nws = int(lib.vsiq_pcm_workspace_doubles(H.c_i64(rows), H.c_i64(rowlen)))
    ws = torch.zeros(max(nws, 1), dtype=torch.float64, device=dev)
    gsc = torch.empty(rows, dtype=torch.float64, device=dev)
    gzp = torch.empty(rows, dtype=torch.float64, device=dev)

    def k6(i):
        j = i % sl
        return lib.vsiq_pcm_lsq_bwd_f32(P(gs[j].data_ptr()), P(xs[j].data_ptr()), P(gxs[j].data_ptr()),
                                        H.c_i64(rows), H.c_i64(rowlen), H.c_i64(rows), P(sc.data_ptr()),
                                        P(zp.data_ptr()), 1, -128, 127, 1e-4, P(gsc.data_ptr()), P(gzp.data_ptr()),
                                        P(ws.data_ptr()), H.c_i64(nws), st)

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
    print(" gate   K3 us  STE us  plain us  pcm us  pcm+mask us  K6 us")
    try:
        for gt in gates:
            H.set_tuning(H.TUNE_STORE_GATE, gt)
            a = t(k3)
            c = t(ste)
            b = t(plain(gt))
            d = t(pcm(False))
            e = t(pcm(True))
            f = t(k6)
            res.append((gt, a, b, c, d, e, f))
            print(f"{gt:5d} {a:7.2f} {c:7.2f} {b:9.2f} {d:7.2f} {e:11.2f} {f:6.2f}", flush=True)
    finally:
        H.set_tuning(H.TUNE_STORE_GATE, -1)
    pa = min(res, key=lambda r: r[2])
    print(f"best plain copy {pa[2]:.2f} us at gate {pa[0]} = {alg / pa[2] / 1e3:.0f} GB/s ({alg / pa[2] / 8e6:.3f} of 8 TB/s)")
    for name, col in (("K3", 1), ("STE", 3), ("pcm fwd", 4), ("pcm fwd + mask", 5), ("K6", 6)):
        ka = min(res, key=lambda r: r[col])
        nb = alg * 3 // 2 if col == 6 else alg
        print(f"best {name} {ka[col]:.2f} us at gate {ka[0]} = {nb / ka[col] / 1e3:.0f} GB/s "
              f"({nb / ka[col] / 8e6:.3f} of 8 TB/s); no gate {res[0][col]:.2f} us")


if __name__ == "__main__":
    main()
