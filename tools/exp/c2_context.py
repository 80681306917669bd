"""C2's kernels in the bench's context rather than back to back: groups of G forwards (K3,
vsiq_pc_observe_fq_f32) then G STE backwards (vsiq_ste_bwd_f32) over 8 rotated buffers,
HIP events around each phase exactly as bench.py's C2PerChannel.launch_group, with each
kernel's store gate forced per phase (VSIQ_TUNE_STORE_GATE set between the phases).

For G in GROUPS and a sweep of one kernel's gate (the other at a fixed gate) prints the
us per launch of each phase, so that (a) the cost of the phase transition (G = 8 against
G = 64) and (b) the gate optimum in context (against c2_floor.py's back-to-back optimum)
can be read off.
usage: python tools/exp/c2_context.py [rounds]"""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from vsiquantization_amd import _hip as H  # noqa: E402
from vsiquantization_amd.fakequant import qden  # noqa: E402
import bench  # noqa: E402

P = ctypes.c_void_p


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 25
    dev = torch.device("cuda:0")
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    lib = H.lib()
    st = H.stream_of(dev)
    rows, rowlen, sl = 1024, 9216, 8
    g = torch.Generator(device=dev).manual_seed(0)
    xs = [torch.randn(rows, rowlen, device=dev, generator=g) * 0.05 for _ in range(sl)]
    ys = [torch.empty_like(xs[0]) for _ in range(sl)]
    gs = [torch.randn(rows, rowlen, device=dev, generator=g) for _ in range(sl)]
    gxs = [torch.empty_like(xs[0]) for _ in range(sl)]
    mw = int(lib.vsiq_mask_words(H.c_i64(rows), H.c_i64(rowlen)))
    masks = [torch.empty(mw, dtype=torch.int64, device=dev) for _ in range(sl)]
    run = [torch.zeros(2, rows, device=dev) for _ in range(sl)]
    qp = [torch.empty(2, rows, dtype=torch.float64, device=dev) for _ in range(sl)]
    qd = qden(False, 8, 1e-8)
    if os.environ.get("SHARED", "0") == "1":   # one mask / state for all slots (c2_floor.py's setup)
        masks, run, qp = [masks[0]] * sl, [run[0]] * sl, [qp[0]] * sl
    fwd = [(P(xs[j].data_ptr()), P(ys[j].data_ptr()), None, P(masks[j].data_ptr()), H.c_i64(rows),
            H.c_i64(rowlen), P(run[j][0].data_ptr()), P(run[j][1].data_ptr()), P(qp[j][0].data_ptr()),
            P(qp[j][1].data_ptr()), None, 0, 0, 255, qd, 1e-8, st) for j in range(sl)]
    bwd = [(P(gs[j].data_ptr()), P(masks[j].data_ptr()), P(gxs[j].data_ptr()), H.c_i64(rows * rowlen),
            P(qp[j][0].data_ptr()), H.c_i64(rowlen), 0.0, st) for j in range(sl)]
    f_fwd, f_bwd = lib.vsiq_pc_observe_fq_f32, lib.vsiq_ste_bwd_f32
    partner = os.environ.get("PARTNER", "ste")   # what runs between the K3 phases
    if partner == "copy":   # a plain ungated copy of the STE's bytes (c2_floor.hip)
        import subprocess
        so = os.path.join("/tmp", "c2_floor.so")
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-o", so,
                        os.path.join(HERE, "c2_floor.hip")], check=True)
        ex = ctypes.CDLL(so)
        ex.exp_copy_gated.argtypes = [P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint32, P]
        f_bwd = lambda a, b, c, *_: ex.exp_copy_gated(a, c, rows, rowlen, 0, st)   # noqa: E731
    elif partner == "tiny":   # a one-workgroup kernel: no traffic
        tiny = torch.empty(64, device=dev)
        f_bwd = lambda *_: (tiny.fill_(0.0), 0)[1]   # noqa: E731
    elif partner == "ste_ownmask":   # the STE on masks K3 never writes (same bytes)
        own = [m.clone() for m in masks]
        bwd = [(b[0], P(own[j].data_ptr()), *b[2:]) for j, b in enumerate(bwd)]

    def run_groups(G, gk3, gste):
        """rounds x (G fwds, G bwds); returns (us per K3, us per STE): median over rounds."""
        evs = [[bench.timing_event() for _ in range(3)] for _ in range(rounds + 2)]
        one = os.environ.get("ONEGATE", "0") == "1"   # both kernels at gk3, no switch per phase
        if one:
            H.set_tuning(H.TUNE_STORE_GATE, gk3)
        for r, ev in enumerate(evs):
            if not one:
                H.set_tuning(H.TUNE_STORE_GATE, gk3)
            ev[0].record()
            for j in range(G):
                f_fwd(*fwd[j % sl])
            ev[1].record()
            if not one:
                H.set_tuning(H.TUNE_STORE_GATE, gste)
            for j in range(G):
                f_bwd(*bwd[j % sl])
            ev[2].record()
        torch.cuda.synchronize()
        a = sorted(e[0].elapsed_time(e[1]) * 1e3 / G for e in evs[2:])
        b = sorted(e[1].elapsed_time(e[2]) * 1e3 / G for e in evs[2:])
        return a[len(a) // 2], b[len(b) // 2]

    gates = [0] + list(range(453, 623, 13))
    if os.environ.get("NT", "1") == "0":
        H.set_tuning(H.TUNE_NONTEMPORAL, 0)
    glist = [int(v) for v in os.environ.get("CTX_GROUPS", "8,64").split(",")]
    if os.environ.get("K3ONLY", "0") == "1":   # K3 back to back, timed per 64 launches
        try:
            for gt in gates:
                H.set_tuning(H.TUNE_STORE_GATE, gt)
                for j in range(16):
                    f_fwd(*fwd[j % sl])
                evs = [(bench.timing_event(), bench.timing_event()) for _ in range(rounds)]
                for e0, e1 in evs:
                    e0.record()
                    for j in range(64):
                        f_fwd(*fwd[j % sl])
                    e1.record()
                torch.cuda.synchronize()
                a = sorted(e0.elapsed_time(e1) * 1e3 / 64 for e0, e1 in evs)
                print(f"{gt:5d} K3 only {a[len(a) // 2]:7.2f}", flush=True)
        finally:
            H.set_tuning(H.TUNE_STORE_GATE, -1)
        return
    try:
        for G in glist:
            run_groups(G, 500, 0)
            print(f"G={G}: K3 gate sweep (STE gate 0)        |  STE gate sweep (K3 gate 492)")
            print(" gate   K3 us  (STE us)  |  STE us  (K3 us)")
            for gt in gates:
                a, b = run_groups(G, gt, 0)
                c, d = run_groups(G, 492, gt)
                print(f"{gt:5d} {a:7.2f} ({b:6.2f})  | {d:7.2f} ({c:6.2f})", flush=True)
    finally:
        H.set_tuning(H.TUNE_STORE_GATE, -1)


if __name__ == "__main__":
    main()
