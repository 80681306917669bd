"""K2o (vsiq_act_observe_part_out_f32, calibrate_qat_model's default per-layer pass) on
the C5 workload: the YOLOv8n backbone's 27 fused-ReLU layers at 128 images, one launch
per layer in layer order (what _observe_deferred_act issues), against

  * the activation alone (vsiq_act_fwd_f32: the same 1:1 stream without the observer),
  * K2p alone (vsiq_act_observe_part_f32: the observer without the y stores),
  * the grid-stride K2o form (VSIQ_TUNE_K2O_FORM 1, round 3's kernel),
  * every one-shot groups-per-lane instance (VSIQ_TUNE_K2O_GROUPS).

Phase time by HIP events (hipEventDisableSystemFence) around R repetitions of the
27-launch phase, algorithmic bytes 8 B/elem (K2p 4 B/elem).  Run under
`rocprofv3 --kernel-trace --stats` for per-launch durations by layer size.
usage: python tools/exp/k2o_bench.py [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vsiquantization_amd import _hip as H  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    lib = H.lib()
    st = H.stream_of(dev)
    gen = torch.Generator(device=dev).manual_seed(5)
    acts = [torch.randn(128, co, h, h, device=dev, generator=gen) for _, co, _, _, h in bench.yolov8n_backbone()]
    ys = [torch.empty_like(a) for a in acts]
    n = sum(a.numel() for a in acts)
    slot = torch.empty((1 << 16) * H.PART_LEN, dtype=torch.float64, device=dev)   # G=1 at 52M: 51200 records
    relu = H.ACT_RELU

    def k2o():
        for a, y in zip(acts, ys):
            assert lib.vsiq_act_observe_part_out_f32(H.ptr(a), H.ptr(y), H.c_i64(a.numel()), relu, H.ptr(slot),
                                                     H.c_i64(slot.numel()), st) == 0

    def act_only():
        for a, y in zip(acts, ys):
            assert lib.vsiq_act_fwd_f32(H.ptr(a), H.ptr(y), H.c_i64(a.numel()), relu, st) == 0

    def k2p():
        for a in acts:
            assert lib.vsiq_act_observe_part_f32(H.ptr(a), H.c_i64(a.numel()), relu, H.ptr(slot),
                                                 H.c_i64(slot.numel()), st) == 0

    def timed(fn, bytes_per_elem):
        for _ in range(3):
            fn()
        e0, e1 = bench.HipEvent(), bench.HipEvent()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        return us, bytes_per_elem * n / us / 1e3

    rows = []
    rows.append(("act only (vsiq_act_fwd_f32)", *timed(act_only, 8)))
    rows.append(("K2p only (read)", *timed(k2p, 4)))
    variants = [(1, 0, 0), (0, 0, 0)] + [(0, g, bs) for bs in (256, 512, 1024) for g in (1, 2, 4)]
    for form, g, bs in variants:
        assert lib.vsiq_set_tuning(H.TUNE_K2O_FORM, form) == 0
        assert lib.vsiq_set_tuning(H.TUNE_K2O_GROUPS, g) == 0
        assert lib.vsiq_set_tuning(H.TUNE_K2O_BLOCK, bs) == 0
        name = "K2o grid-stride (round 3)" if form else f"K2o one-shot G={g or 'dflt'} BS={bs or 'dflt'}"
        rows.append((name, *timed(k2o, 8)))
    for key in (H.TUNE_K2O_FORM, H.TUNE_K2O_GROUPS, H.TUNE_K2O_BLOCK):
        assert lib.vsiq_set_tuning(key, 0) == 0
    # the sync's fold over a calibration run's slots (16 batches x 27 layers, default K2o)
    from vsiquantization_amd.fakequant import fold_parts, part_out_slot_doubles
    stride = max(part_out_slot_doubles(a.numel()) for a in acts)
    slots = torch.zeros(16, len(acts), stride, dtype=torch.float64, device=dev)
    for b in range(16):
        for j, (a, y) in enumerate(zip(acts, ys)):
            assert lib.vsiq_act_observe_part_out_f32(H.ptr(a), H.ptr(y), H.c_i64(a.numel()), relu,
                                                     slots[b, j].data_ptr(), H.c_i64(stride), st) == 0
    flat = slots.reshape(16 * len(acts), stride)
    fold_parts(flat)
    e0, e1 = bench.HipEvent(), bench.HipEvent()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(5):
        fold_parts(flat)
    e1.record()
    torch.cuda.synchronize()
    print(f"sync fold of 16 x 27 default K2o slots ({stride // 8} records max, "
          f"{flat.numel() * 8 / 2**20:.0f} MB of slots): {e0.elapsed_time(e1) * 1e3 / 5:.1f} us")
    print(f"C5 phase: 27 fused-ReLU layers, batch 128, {n / 1e6:.1f}M elements, {reps} reps")
    for name, us, gbs in rows:
        print(f"{name:34s} {us:9.1f} us/phase  {gbs:8.1f} GB/s  frac {gbs / 8000:.3f}")
    print("default records per layer:", [int(lib.vsiq_observe_part_out_records(H.c_i64(a.numel()))) for a in acts])


if __name__ == "__main__":
    main()
