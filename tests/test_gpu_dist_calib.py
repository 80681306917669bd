"""Batch-sharded calibration through the kernels, 2 ranks: per-tensor
activation observers (QuantizationManager, fused ReLU) with an all-reduce of their
statistics -- per call (K2 + finalize) and deferred (K2p records + one sync_calibration)
-- give the 1-GPU min/max and qparams bit for bit and mean|x| / mean / std within 1e-6
(observers/minmax.py:32-74, quantization_manager.py:55-71), including a call whose NaN
sits on one rank only; the 1-GPU run itself equals the oracle (observe_minmax /
minmax_qparams replayed call by call: bitwise; collect_stats: 1e-6).  Configurations
(tests/dist_calib_common.py): "small" (3 layers x 5 calls) and "c5" (C5's structure: the
27 backbone activation quantizers with ReLU x 16 calls of uint8/255-derived inputs, at 4
images per call).  The ranks run as a child torch.distributed.run job (gloo, both on
cuda:0: the collective is RCCL on a real multi-GPU node, the arithmetic around it is
the same).  test_c5_one_batch_full_size: one calibration batch of C5's 128 images per
GPU through the 27 deferred observers against the oracle."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import fakequant_np as O
from tests.dist_calib_common import DEV, Config, activations, managers, observe, state

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle(cfg, acts):
    """Per layer: the reference observer replayed over the calls (minmax.py:32-74, the
    manager's observer is 8-bit symmetric: SURVEY §0.5) and the per-call statistics."""
    from vsiquantization_amd import _hip as H
    out = []
    for li, (act, _) in enumerate(cfg.layers):
        mn, mx, stats = 0, 0, []
        for row in acts:
            a = O.act_forward(row[li].cpu().numpy(), act, H.silu_reference())
            mn, mx = O.observe_minmax(a, mn, mx)
            stats.append(O.collect_stats(a))
        s, z = O.minmax_qparams(mn, mx, True, 8)
        out.append(dict(min=float(mn), max=float(mx), scale=float(s), zp=float(z),
                        mean_abs=[t[0] for t in stats], mean=[t[1] for t in stats], std=[t[2] for t in stats]))
    return out


def _same(got, want, what):
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert (g["min"], g["max"], g["scale"], g["zp"]) == (w["min"], w["max"], w["scale"], w["zp"]), (what, i)
        for k in ("mean_abs", "mean", "std"):
            # the signed mean of zero-centred data cancels: 1e-6 of mean|x| absolute as well
            atol = 1e-6 * max(abs(v) for v in w["mean_abs"] if v == v) if k == "mean" else 1e-12
            np.testing.assert_allclose(g[k], w[k], rtol=1e-6, atol=atol, err_msg=f"{what} layer {i} {k}")


@pytest.mark.parametrize("name,backend,ranks", [("small", "gloo", 2), ("c5", "gloo", 2), ("small", "nccl", 1)])
def test_sharded_calibration_two_ranks_equals_one_gpu(tmp_path, name, backend, ranks):
    """gloo: 2 ranks sharing cuda:0.  nccl: ONE rank over RCCL (two ranks cannot share a
    GPU under RCCL): the RCCL all_gather_into_tensor / all_reduce branches and a
    GraphedStep capture of the per-call observe+quantize step holding an RCCL all_gather."""
    cfg = Config(name)
    out = tmp_path / "rank0.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_calib_worker.py"), str(out), name]
    env = dict(os.environ, VSIQ_DIST_BACKEND=backend)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = json.loads(out.read_text())
    acts = activations(cfg)
    mgrs = managers(cfg)
    observe(cfg, mgrs, acts)
    one = state(mgrs)
    assert len(one[0]["mean_abs"]) == cfg.calls and len(one) == len(cfg.layers)
    _same(one, _oracle(cfg, acts), "1 GPU vs oracle")
    for mode in ("per_call", "deferred"):
        _same(got[mode], one, f"{ranks} ranks ({backend}) {mode} vs 1 GPU")
    assert got["deferred_read_raises"] is True   # a read before sync_calibration, every rank
    if backend == "nccl":
        assert got["graph"]["replays_equal_eager"], got["graph"]
    if name == "small":
        # observe + quantize per call: the 2 ranks' y / straight-through gradients are the
        # 1-GPU run's halves bit for bit, the observer state identical (one all_gather
        # per call, folded inside the fake-quant launch: vsiq_act_fq_fwd_ranks_f32)
        from tests.dist_calib_common import observe_quantize
        mgrs = managers(cfg)
        for qm in mgrs:
            qm.is_quantize = True
        full = observe_quantize(cfg, mgrs, acts)
        _same(got["observe_quantize"], state(mgrs), "2 ranks observe+quantize vs 1 GPU")
        for r in range(ranks):
            part = np.load(f"{out}.oq{r}.npz")
            for k, v in full.items():
                want = np.array_split(v, ranks, axis=0)[r]
                assert np.array_equal(part[k].view(np.uint32), want.view(np.uint32)), (r, k)


def test_c5_one_batch_full_size():
    """C5 per GPU: one calibration batch of 128 images (3x320x320 network input; 274M
    activation elements over the 27 layers) through the deferred observers -- the
    default path of calibrate_qat_model: each fused-ReLU call goes to K2o
    (QuantizationManager._observe_deferred_act -> fakequant.observe_parts_out, which also
    writes ReLU(x)), then one sync -- against the oracle."""
    import bench
    from vsiquantization_amd.distributed import sync_calibration
    cfg = Config("c5")
    cfg.calls, cfg.batch = 1, 128
    gen = torch.Generator(device=DEV)
    acts = [[]]
    for li, (_, shp) in enumerate(cfg.layers):
        gen.manual_seed(77 + li)
        u8 = torch.randint(0, 256, (cfg.batch, *shp), device=DEV, dtype=torch.uint8, generator=gen)
        acts[0].append((u8.float() / 255.0 - 0.45) * (0.5 + 0.25 * (li % 7)))
    assert sum(a.numel() for a in acts[0]) == 128 * 2_137_600 == 128 * sum(
        co * h * h for _, co, _, _, h in bench.yolov8n_backbone())
    mgrs = managers(cfg)
    for qm in mgrs:
        qm.dist_defer = True
    observe(cfg, mgrs, acts)
    sync_calibration(torch.nn.ModuleList(mgrs))
    _same(state(mgrs), _oracle(cfg, acts), "C5 batch 128 vs oracle")


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("act", [None, "relu", "silu"])
def test_ranks_fold_fq_equals_finalize_then_fq(world, act):
    """K1r (vsiq_act_fq_fwd_ranks_f32): the gathered records folded inside the fake-quant
    launch == vsiq_observe_finalize_ranks then K1 on its qparams record, bit for bit
    (running state, qparams record, stats record, y, 1-bit mask), over a state carried
    across calls and a call whose NaN sits on one rank only."""
    from vsiquantization_amd import _hip as H
    from vsiquantization_amd import fakequant as FQ
    gen = torch.Generator(device=DEV).manual_seed(world)
    ra, rb = torch.zeros(2, device=DEV), torch.zeros(2, device=DEV)
    for call in range(3):
        shards = [torch.randn(3 * 40_000 + 17 * r, device=DEV, generator=gen) * (1 + call) for r in range(world)]
        if call == 1:
            shards[-1][5] = float("nan")
        recs = [FQ.observe_tensor(x, symmetric=False, want_qp=False, act=act)[1] for x in shards]
        gathered = torch.cat(recs)
        for r, x in enumerate(shards):
            # finalize + K1 (round 2) on rank r's shard
            st_a = torch.empty(H.ST_LEN, dtype=torch.float64, device=DEV)
            qp_a = torch.empty(H.QP_LEN, dtype=torch.float64, device=DEV)
            run_a = ra.clone()
            H.check(H.lib().vsiq_observe_finalize_ranks(H.ptr(gathered), world, H.ptr(st_a), H.ptr(run_a), H.ptr(qp_a),
                                                        0, FQ.qden(False, 8, 1e-8), 1e-8,
                                                        H.stream_of(torch.device(DEV))), "finalize")
            y_a, m_a, _ = FQ.fake_quant(x, None, None, 0, 255, qp=qp_a, want_mask=True, act=act)
            # K1r
            st_b = torch.empty_like(st_a)
            qp_b = torch.empty_like(qp_a)
            run_b = rb.clone()
            y_b = torch.empty_like(x)
            m_b = H.mask_buffer(1, x.numel(), x.device)
            H.check(H.lib().vsiq_act_fq_fwd_ranks_f32(H.ptr(x), H.ptr(y_b), None, H.ptr(m_b), H.c_i64(x.numel()),
                                                      H.act_code(act), H.ptr(gathered), world, H.ptr(st_b),
                                                      H.ptr(run_b), H.ptr(qp_b), 0, FQ.qden(False, 8, 1e-8), 1e-8,
                                                      0, 255, H.stream_of(torch.device(DEV))), "ranks fq")
            for u, v in ((run_a, run_b), (qp_a, qp_b), (y_a, y_b), (m_a, m_b)):
                assert torch.equal(u.view(torch.int32 if u.dtype == torch.float32 else torch.int64),
                                   v.view(torch.int32 if v.dtype == torch.float32 else torch.int64)), (call, r)
            assert torch.equal(st_a.view(torch.int64), st_b.view(torch.int64)), (call, r)
        ra, rb = run_a, run_b


def test_sharded_silu_follows_each_ranks_layout():
    """Sharded fused SiLU (distributed.py:10-11): under the reference's DDP every rank runs
    F.silu on its own shard, so rank r's activation is torch CPU silu over THAT shard's
    layout (fused.py:133).  Pinned here on ragged shards of 3 ranks through K2 records +
    K1r: each rank's y and mask == the oracle's silu of its shard, quantized with the
    qparams of the oracle's running min/max over all shards' outputs (bitwise).  Against a
    1-GPU whole-batch run (itself == the oracle over the whole batch) the activations may
    differ only at elements whose exp path (Sleef vector / glibc scalar) the two layouts
    choose differently."""
    from vsiquantization_amd import _hip as H
    from vsiquantization_amd import fakequant as FQ
    from tests import goldens as G
    ref = (32, 8)
    H.set_silu_reference(*ref)
    try:
        sizes = [40_001, 39_993, 40_027]
        gen = torch.Generator(device=DEV).manual_seed(5)
        whole = torch.randn(sum(sizes), device=DEV, generator=gen) * 4
        shards = list(torch.split(whole, sizes))
        a_sh = [O.silu_forward(x.cpu().numpy(), ref) for x in shards]
        mn, mx = O.observe_minmax(np.concatenate(a_sh))
        s, z = O.minmax_qparams(mn, mx, True, 8)
        recs = [FQ.observe_tensor(x, symmetric=True, want_qp=False, act="silu")[1] for x in shards]
        gathered = torch.cat(recs)
        st = H.stream_of(torch.device(DEV))
        for r, x in enumerate(shards):
            run = torch.zeros(2, device=DEV)
            qp = torch.empty(H.QP_LEN, dtype=torch.float64, device=DEV)
            stats = torch.empty(H.ST_LEN, dtype=torch.float64, device=DEV)
            y = torch.empty_like(x)
            m = H.mask_buffer(1, x.numel(), x.device)
            H.check(H.lib().vsiq_act_fq_fwd_ranks_f32(
                H.ptr(x), H.ptr(y), None, H.ptr(m), H.c_i64(x.numel()), H.act_code("silu"), H.ptr(gathered),
                len(shards), H.ptr(stats), H.ptr(run), H.ptr(qp), 1, FQ.qden(True, 8, 1e-8), 1e-8, -128, 127, st),
                "ranks fq")
            assert (float(run[0]), float(run[1])) == (mn, mx), r
            assert (float(qp[H.QP_SCALE]), float(qp[H.QP_ZP])) == (s, z), r
            yo, _, mo = O.fq_forward(a_sh[r], s, z, -128, 127)
            assert np.array_equal(y.cpu().numpy().view(np.uint32), yo.view(np.uint32)), r
            assert np.array_equal(G.unpack_mask(m.cpu().numpy(), 1, x.numel())[0], mo), r
        # the 1-GPU whole batch: its own layout, == the oracle; differences to the shards'
        # activations only where the exp path differs between the two layouts
        y1 = FQ.activation(whole, "silu").cpu().numpy()
        a1 = O.silu_forward(whole.cpu().numpy(), ref)
        assert np.array_equal(y1.view(np.uint32), a1.view(np.uint32))
        a_cat = np.concatenate(a_sh)
        path_diff = O.silu_scalar_map(whole.numel(), ref) != np.concatenate(
            [O.silu_scalar_map(n, ref) for n in sizes])
        assert path_diff.any()
        assert not (a_cat.view(np.uint32) != a1.view(np.uint32))[~path_diff].any()
    finally:
        H.set_silu_reference()
