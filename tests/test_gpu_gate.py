"""Store-gate tuner (csrc/gate_tune.hip, VSIQ_TUNE_GATE_AUTOTUNE): the first launches of
a one-round launch site run candidate gates, timed by event pairs; the gate is a pure
delay, so every candidate must give the same bits.  C2-shaped K3 forward and STE
backward run through tuning and are compared with the oracle (bitwise) at every launch;
the tuner must settle and report the sites."""
import numpy as np
import pytest
import torch

from vsiquantization_amd import _hip as H
from vsiquantization_amd import fakequant as FQ
from oracle import fakequant_np as O
from tests import goldens as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _reset():
    torch.cuda.synchronize()
    assert H.lib().vsiq_gate_reset() == 0


@pytest.mark.parametrize("shape", [(1024, 1024, 3, 3), (768, 512, 3, 3)])
def test_tuned_gate_bits_identical_to_oracle(shape):
    rng = np.random.default_rng(5)
    w = (rng.standard_normal(shape) * 0.05).astype(np.float32)
    g = rng.standard_normal(shape).astype(np.float32)
    ref = O.per_channel_observe_fq(w, False, 8)
    gxo = O.per_channel_backward_fixed(g, ref["mask"], ref["scale"])
    x, gd = torch.from_numpy(w).to(DEV), torch.from_numpy(g).to(DEV)
    rowlen = w.size // shape[0]
    _reset()
    ys, gxs = [], []
    for i in range(600):   # > 12 candidates x 8 samples + 3 finalists x 8 more, per site (x4 if bursts)
        r = FQ.per_channel_observe_fq(x, symmetric=False, qmin=0, qmax=255, want_mask=True)
        gx = FQ.ste_backward(gd, r["mask"], r["scale"], rowlen)
        if i % 29 == 0:
            ys.append(r["y"].clone())
            gxs.append(gx.clone())
        if i % 16 == 15:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    for y, gx in zip(ys, gxs):
        G.assert_bitwise_f32(y.cpu().numpy(), ref["y"], "y")
        G.assert_bitwise_f32(gx.cpu().numpy(), gxo, "grad_x")
    assert H.gate_tuning_pending() == 0
    rep = H.gate_report()
    lines = {l.split()[0]: l for l in rep.splitlines()}
    sites = ("k3_pc_observe_fq", "ste_bwd") if shape[1] * shape[2] * shape[3] == 9216 else ("k3_pc_observe_fq",)
    for k in sites:   # the STE grid of 4608-element rows is not a one-round 9-group grid
        assert k in lines, rep
        assert " done=1 " in lines[k], rep
        assert f"grid={shape[0]} " in lines[k], rep


def test_forced_gate_and_autotune_off():
    """VSIQ_TUNE_STORE_GATE forces ticks (no tuning); GATE_AUTOTUNE 0 keeps the fixed
    estimate and creates no site."""
    x = torch.randn(1024, 9216, device=DEV) * 0.05
    _reset()
    try:
        H.set_tuning(H.TUNE_GATE_AUTOTUNE, 0)
        y0 = FQ.per_channel_observe_fq(x, symmetric=False, qmin=0, qmax=255)["y"]
        H.set_tuning(H.TUNE_STORE_GATE, 700)
        y1 = FQ.per_channel_observe_fq(x, symmetric=False, qmin=0, qmax=255)["y"]
        torch.cuda.synchronize()
        assert H.gate_report() == ""
        assert torch.equal(y0.view(torch.int32), y1.view(torch.int32))
    finally:
        H.set_tuning(H.TUNE_GATE_AUTOTUNE, 1)
        H.set_tuning(H.TUNE_STORE_GATE, -1)


def test_capture_uses_current_gate_and_matches_eager():
    """A launch under HIP-graph capture is never timed; replay == eager bit for bit."""
    x = torch.randn(1024, 9216, device=DEV) * 0.05
    _reset()
    eager = FQ.per_channel_observe_fq(x, symmetric=False, qmin=0, qmax=255)["y"].clone()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            out = FQ.per_channel_observe_fq(x, symmetric=False, qmin=0, qmax=255)["y"]
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), eager.view(torch.int32))


def _site_line(name):
    return {l.split()[0]: l for l in H.gate_report().splitlines()}.get(name, "")


def _retunes(line):
    return int(line.split("retunes=")[1].split()[0]) if "retunes=" in line else -1


def _k3_inputs():
    rng = np.random.default_rng(9)
    w = (rng.standard_normal((1024, 1024, 3, 3)) * 0.05).astype(np.float32)
    return torch.from_numpy(w).to(DEV), O.per_channel_observe_fq(w, False, 8)["y"]


def test_gate_retune_api_retunes_every_site_bits_identical():
    """vsiq_gate_retune: every site tunes again from its next launches (under the load of
    the moment); the outputs stay bit-identical throughout."""
    x, want = _k3_inputs()
    _reset()
    for _ in range(600):
        FQ.per_channel_observe_fq(x, symmetric=False, qmin=0, qmax=255)
    torch.cuda.synchronize()
    assert H.gate_tuning_pending() == 0 and " done=1 " in _site_line("k3_pc_observe_fq")
    assert H.gate_retune() >= 1
    assert " done=0 " in _site_line("k3_pc_observe_fq")
    ys = []
    for i in range(600):
        y = FQ.per_channel_observe_fq(x, symmetric=False, qmin=0, qmax=255)["y"]
        if i % 10 == 0:
            ys.append(y.clone())
        if i % 16 == 15:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    line = _site_line("k3_pc_observe_fq")
    assert " done=1 " in line and _retunes(line) >= 1, line
    for y in ys:
        G.assert_bitwise_f32(y.cpu().numpy(), want, "y")


def _k3_direct(x):
    """K3 through the C ABI with preallocated outputs: launches enqueue faster than they
    run (a Python-level call allocating its outputs leaves the GPU idle between launches,
    and the tuner's event pairs then time the launch latency too)."""
    from vsiquantization_amd.fakequant import qden
    rows, rowlen = x.shape[0], x.numel() // x.shape[0]
    y = torch.empty_like(x)
    mask = torch.empty(int(H.lib().vsiq_mask_words(H.c_i64(rows), H.c_i64(rowlen))), dtype=torch.int64, device=DEV)
    run = torch.zeros(2, rows, device=DEV)
    qp = torch.empty(2, rows, dtype=torch.float64, device=DEV)
    st = H.stream_of(torch.device(DEV))
    args = (H.ptr(x), H.ptr(y), None, H.ptr(mask), H.c_i64(rows), H.c_i64(rowlen), H.ptr(run[0]), H.ptr(run[1]),
            H.ptr(qp[0]), H.ptr(qp[1]), None, 0, 0, 255, qden(False, 8, 1e-8), 1e-8, st)

    def launch():
        assert H.lib().vsiq_pc_observe_fq_f32(*args) == 0
        return y
    return launch


def test_gate_drift_under_concurrent_load_retunes():
    """A tuned site times one launch in 128; two concurrent streams streaming HBM copies
    slow the launches by far more than 15 % for two drift checks in a row (2 x 8 samples,
    about 2048 launches), so the site re-tunes by itself; the outputs stay bit-identical."""
    x, want = _k3_inputs()
    launch = _k3_direct(x)
    _reset()
    for i in range(800):   # back to back: bursts of 4 launches per sample
        launch()
        if i % 16 == 15:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    line0 = _site_line("k3_pc_observe_fq")
    assert " done=1 " in line0 and _retunes(line0) == 0, line0
    loads = [(torch.empty(1 << 28, device=DEV), torch.empty(1 << 28, device=DEV), torch.cuda.Stream())
             for _ in range(2)]   # 1 GiB each way per stream
    ys = []
    for rnd in range(12):
        for a, b, st in loads:
            with torch.cuda.stream(st):
                for _ in range(60):
                    b.copy_(a)
        for i in range(400):
            y = launch()
            if i % 100 == 0:
                ys.append(y.clone())
        torch.cuda.synchronize()
        if _retunes(_site_line("k3_pc_observe_fq")) >= 1:
            break
    line = _site_line("k3_pc_observe_fq")
    assert _retunes(line) >= 1, (line0, line)
    for y in ys:
        G.assert_bitwise_f32(y.cpu().numpy(), want, "y")


def test_burst_sample_never_spans_another_library_launch():
    """A site's burst sample ends at any other launch of the library (g_lib_launches): a
    1.6M-element K2o (a one-round gated site) alternating with a 52M-element K2o (an
    untuned multi-round grid, ~70 us) -- were a sample to span the large launch, every
    candidate's median would carry it.  The outputs stay the oracle's ReLU bits."""
    _reset()
    small = torch.randn(1_638_400, device=DEV)
    big = torch.randn(52_428_800, device=DEV)
    for i in range(400):
        y, _ = FQ.observe_parts_out(small, "relu")
        FQ.observe_parts_out(big, "relu")
        if i % 16 == 15:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    G.assert_bitwise_f32(y.cpu().numpy(), O.act_forward(small.cpu().numpy(), "relu"), "relu")
    line = _site_line("k2o_observe_out")
    assert " done=1 " in line, H.gate_report()
    meds = [float(t.split(":")[1]) for t in line.split() if ":" in t and t.split(":")[0].isdigit()]
    assert len(meds) >= 12 and max(meds) < 30.0, line


def test_burst_sample_excludes_foreign_kernels():
    """Kernels of another library (here torch's elementwise add over 52M floats, ~70 us)
    queued between two launches of a burst are not counted: every launch of a burst has
    its own event pair (round 6).  K3 at C2 through the C ABI (launches enqueue within the
    burst gap) alternates with the torch op; every candidate's median stays a K3 time."""
    x, want = _k3_inputs()
    launch = _k3_direct(x)
    big = torch.zeros(52_428_800, device=DEV)
    _reset()
    for i in range(800):
        y = launch()
        big.add_(1.0)
        if i % 16 == 15:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    G.assert_bitwise_f32(y.cpu().numpy(), want, "y")
    line = _site_line("k3_pc_observe_fq")
    assert " done=1 " in line, H.gate_report()
    meds = [float(t.split(":")[1]) for t in line.split() if ":" in t and t.split(":")[0].isdigit()]
    assert len(meds) >= 12 and max(meds) < 40.0, line


def test_gate_table_save_load_freeze(tmp_path):
    """A tuned table saved (vsiq_gate_export), reset, loaded and frozen: every site launched
    again takes its saved gate and is never timed (no candidate medians in the report, no
    drift samples), results stay bitwise, and a site missing from the table runs the fixed
    default without tuning.  Unfreezing restores online tuning."""
    shape = (1024, 1024, 3, 3)
    rng = np.random.default_rng(9)
    w = (rng.standard_normal(shape) * 0.05).astype(np.float32)
    ref = O.per_channel_observe_fq(w, False, 8)
    x = torch.from_numpy(w).to(DEV)
    _reset()
    for i in range(600):
        FQ.per_channel_observe_fq(x, symmetric=False, qmin=0, qmax=255)
        if i % 16 == 15:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    assert H.gate_tuning_pending() == 0
    path = str(tmp_path / "gates.txt")
    nsaved = H.gate_save(path)
    saved = {l.rsplit(" ", 1)[0]: int(l.rsplit(" ", 1)[1]) for l in open(path).read().splitlines()}
    assert nsaved >= 1 and any("k_pc_observe_fq" in k for k in saved)
    _reset()
    try:
        assert H.gate_load(path) == nsaved
        for i in range(200):
            y = FQ.per_channel_observe_fq(x, symmetric=False, qmin=0, qmax=255)["y"]
        # a different grid (768 rows): not in the table -> the fixed default, untimed
        x2 = torch.from_numpy((rng.standard_normal((768, 512, 3, 3)) * 0.05).astype(np.float32)).to(DEV)
        for i in range(50):
            FQ.per_channel_observe_fq(x2, symmetric=False, qmin=0, qmax=255)
        torch.cuda.synchronize()
        G.assert_bitwise_f32(y.cpu().numpy(), ref["y"], "y (frozen table)")
        assert H.gate_tuning_pending() == 0
        for line in H.gate_report().splitlines():
            f = line.split()
            assert " done=1 " in line and not any(":" in t for t in f[1:]), line   # nothing timed
            if "grid=1024 " in line and f[0] == "k3_pc_observe_fq":
                assert " preset=1 " in line + " ", line
        exported = {l.rsplit(" ", 1)[0]: int(l.rsplit(" ", 1)[1]) for l in H.gate_export().splitlines()}
        for k, v in saved.items():
            assert exported.get(k) == v, (k, v, exported.get(k))
        assert H.gate_retune() == 0   # frozen: nothing re-tunes
    finally:
        H.gate_freeze(False)
        _reset()
