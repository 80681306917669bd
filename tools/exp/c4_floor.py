"""Is C4's records-only backward (K4d: vsiq_act_lsq_bwd_part_f32, fused ReLU, 2 groups per
lane) at the launch floor of its traffic mix?  Per C4 activation size (YOLOv8n backbone at
batch 256): R launches back to back, buffers rotated past the 256 MB MALL, event-timed, of

  * K4d records-only (the product kernel: read g, read c, write grad_c + one record per
    workgroup; 12 B/elem),
  * a plain 2:1 nontemporal streaming kernel with the same access pattern (c4_floor.hip
    exp_add2: y = a + b, one-shot grid) at G = 1 / 2 / 4 / 8 groups per lane.

Prints us per launch, GB/s and K4d / best-plain.  usage: python tools/exp/c4_floor.py"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vsiquantization_amd import _hip as H  # noqa: E402

P = ctypes.c_void_p


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    lib = H.lib()
    ex = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "c4_floor.so"))
    ex.exp_add2.argtypes = [P, P, P, ctypes.c_int64, ctypes.c_int, P]
    st = H.stream_of(dev)
    # C4's activation scale (bench.C4Backbone: 2 * 0.8 / sqrt(qmax), a4): most elements in range
    # (SCALE=0.03: most clamped -- the element math then costs more, profiles/r04f_k4_variants.txt)
    scale = torch.tensor(float(os.environ.get("SCALE", 2 * 0.8 / 7 ** 0.5)), dtype=torch.float64, device=dev)
    sizes = sorted({256 * co * h * h for _, co, _, _, h in bench.yolov8n_backbone()})
    print("C4 act sizes (batch 256), R launches back to back, buffers rotated past the MALL")
    for n in sizes:
        sl = max(2, min(8, (1800 << 20) // (12 * n)))
        gs = [torch.randn(n, device=dev) for _ in range(sl)]
        xs = [torch.randn(n, device=dev) for _ in range(sl)]
        ys = [torch.empty(n, device=dev) for _ in range(sl)]
        nrec = int(lib.vsiq_lsq_part_records(H.c_i64(n)))
        rec = torch.empty(2 * nrec, dtype=torch.float64, device=dev)
        reps = max(20, min(400, (16 << 30) // (12 * n)))

        def k4d(i):
            j = i % sl
            return lib.vsiq_act_lsq_bwd_part_f32(P(gs[j].data_ptr()), P(xs[j].data_ptr()), P(ys[j].data_ptr()),
                                                 H.c_i64(n), H.ACT_RELU, H.ptr(scale), 0.0, None, 0.0, 0, -8, 7,
                                                 H.ptr(rec), H.c_i64(rec.numel()), st)

        def plain(G):
            return lambda i: ex.exp_add2(P(gs[i % sl].data_ptr()), P(xs[i % sl].data_ptr()),
                                         P(ys[i % sl].data_ptr()), n // 4, G, st)

        def t(fn):
            for i in range(8):
                assert fn(i) == 0
            out = []
            for _ in range(3):
                e0, e1 = bench.HipEvent(), bench.HipEvent()
                torch.cuda.synchronize()
                e0.record()
                for i in range(reps):
                    fn(i)
                e1.record()
                torch.cuda.synchronize()
                out.append(e0.elapsed_time(e1) * 1e3 / reps)
            return sorted(out)[1]

        row = {"K4d": t(k4d)}
        for G in (1, 2, 4, 8):
            row[f"2:1 G={G}"] = t(plain(G))
        best = min(v for k, v in row.items() if not k.startswith("K4d"))
        cells = "  ".join(f"{k} {v:8.2f} us {12 * n / v / 1e3:6.0f} GB/s" for k, v in row.items())
        print(f"n={n:10d} {cells}  K4d/best-plain {best / row['K4d']:.3f} (frac K4d {12 * n / row['K4d'] / 8e6:.3f})",
              flush=True)
        del gs, xs, ys
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
