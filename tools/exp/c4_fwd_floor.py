"""C4's forward per activation size: K1 with the fused ReLU (vsiq_act_fq_fwd_f32, learnable
scale on the device, no mask / codes -- the C4 leg's launch) against a plain nontemporal
1:1 y = max(c, 0) kernel with the same access pattern (c4_floor.hip exp_relu1, best of
1/2/4/8 groups per lane), back to back, buffers rotated past the MALL.  8 B/elem.
usage: python tools/exp/c4_fwd_floor.py"""
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
    ex.exp_relu1.argtypes = [P, P, ctypes.c_int64, ctypes.c_int, P]
    st = H.stream_of(dev)
    scale = torch.tensor(2 * 0.8 / 7 ** 0.5, dtype=torch.float64, device=dev)
    sizes = sorted({256 * co * h * h for _, co, _, _, h in bench.yolov8n_backbone()})
    print("C4 act sizes (batch 256), K1-relu fwd vs plain 1:1, R launches back to back, buffers rotated past the MALL")
    for n in sizes:
        sl = max(2, min(8, (1800 << 20) // (8 * n)))
        xs = [torch.randn(n, device=dev) for _ in range(sl)]
        ys = [torch.empty(n, device=dev) for _ in range(sl)]
        reps = max(20, min(400, (16 << 30) // (8 * n)))

        def k1(i):
            j = i % sl
            return lib.vsiq_act_fq_fwd_f32(P(xs[j].data_ptr()), P(ys[j].data_ptr()), None, None, H.c_i64(n),
                                           H.ACT_RELU, None, H.ptr(scale), 0.0, None, 0.0, 0, 0, -8, 7, st)

        def plain(G):
            return lambda i: ex.exp_relu1(P(xs[i % sl].data_ptr()), P(ys[i % sl].data_ptr()), n // 4, G, st)

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

        row = {"K1": t(k1)}
        for G in (1, 2, 4, 8):
            row[f"1:1 G={G}"] = t(plain(G))
        best = min(v for k, v in row.items() if k != "K1")
        cells = "  ".join(f"{k} {v:8.2f} us {8 * n / v / 1e3:6.0f} GB/s" for k, v in row.items())
        print(f"n={n:10d} {cells}  K1/best-plain {best / row['K1']:.3f} (frac K1 {8 * n / row['K1'] / 8e6:.3f})",
              flush=True)
        del xs, ys
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
