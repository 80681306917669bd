"""What the opt-in mean reference (H.set_mean_reference: K11's torch-order mean|x| / mean and
its std pass, per calibration call) costs in C5's calibration batch: per batch of 128
images, the 27 YOLOv8n backbone layers' K2o launches (the default calibration kernel,
through the C ABI as bench.py's C5 leg) alone, and K2o plus fakequant.torch_stats of each
layer's relu(c) (what QuantizationManager._defer_exact adds under the mean reference).
Event-timed over R batches after W warm-up batches.  Experiment only.
usage: python tools/exp/k11_calib_cost.py [R]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vsiquantization_amd import _hip as H  # noqa: E402
from vsiquantization_amd.fakequant import part_out_slot_doubles, torch_stats  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    st = H.stream_of(dev)
    lib = H.lib()
    layers = bench.yolov8n_backbone()
    gen = torch.Generator(device=dev).manual_seed(1)
    acts = [torch.randn(128, co, h, h, device=dev, generator=gen) for _, co, _, _, h in layers]
    ys = [torch.empty_like(a) for a in acts]
    stride = max(part_out_slot_doubles(a.numel()) for a in acts)
    parts = torch.zeros(len(acts), stride, dtype=torch.float64, device=dev)
    n = sum(a.numel() for a in acts)

    def k2o():
        for j, (a, y) in enumerate(zip(acts, ys)):
            rc = lib.vsiq_act_observe_part_out_f32(H.ptr(a), H.ptr(y), H.c_i64(a.numel()), H.ACT_RELU,
                                                   parts[j].data_ptr(), H.c_i64(stride), st)
            assert rc == 0

    def k2o_exact():
        for j, (a, y) in enumerate(zip(acts, ys)):
            rc = lib.vsiq_act_observe_part_out_f32(H.ptr(a), H.ptr(y), H.c_i64(a.numel()), H.ACT_RELU,
                                                   parts[j].data_ptr(), H.c_i64(stride), st)
            assert rc == 0
            torch_stats(a, act="relu", ref=(8, 8))

    def t(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) * 1e3 / reps

    base, ex = t(k2o), t(k2o_exact)
    print(f"C5 batch (27 layers, {n / 1e6:.1f}M elements): K2o only {base:8.1f} us/batch "
          f"({8 * n / base / 1e3:5.0f} GB/s); with the mean reference's torch_stats {ex:8.1f} us/batch "
          f"(+{ex - base:.1f} us, {ex / base:.2f}x; {(ex - base) / len(acts):.1f} us per call)", flush=True)


if __name__ == "__main__":
    main()
