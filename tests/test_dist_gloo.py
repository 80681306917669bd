"""Multi-rank observer reduction on CPU (gloo, world_size 2).

The per-rank statistics records are produced here by the numpy oracle (the K2
kernel needs a GPU); what is tested is the exchange: the all-reduce packing
(MAX over [-min, max], SUM over counts/sums), the fp32-rounded means and the
running-state replay — sharded results must equal the unsharded ones exactly for
min/max/qparams and within 1e-6 for mean|x| / std.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vsiquantization_amd import _hip as H
from vsiquantization_amd.distributed import allreduce_stats, finish_stats, replay_minmax
from oracle import fakequant_np as O


def record(x):
    """Oracle stand-in for one K2 stats record (f64[ST_LEN])."""
    x = np.asarray(x, np.float32)
    r = np.zeros(H.ST_LEN)
    nn = x[~np.isnan(x)]
    r[H.ST_MIN] = nn.min() if nn.size else np.inf
    r[H.ST_MAX] = nn.max() if nn.size else -np.inf
    r[H.ST_NAN] = np.isnan(x).sum()
    d = x.astype(np.float64)
    r[H.ST_SUMABS], r[H.ST_SUM], r[H.ST_SUMSQ], r[H.ST_N] = np.abs(d).sum(), d.sum(), (d * d).sum(), x.size
    return torch.from_numpy(r)


def batches():
    rng = np.random.default_rng(0)
    out = [rng.standard_normal((8, 3, 5, 5)).astype(np.float32) * (1 + i) for i in range(4)]
    out[2][5, 0, 0, 0] = np.nan        # one shard of call 2 holds a NaN: the whole call is skipped
    return out


def _worker(rank, world, port, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        recs = torch.stack([record(np.array_split(b, world)[rank]) for b in batches()])
        red = allreduce_stats(recs.clone())
        ret[rank] = red.numpy().copy()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_observer_matches_single_rank(world):
    port = 29500 + os.getpid() % 1000
    ret = mp.Manager().dict()
    mp.spawn(_worker, args=(world, port, ret), nprocs=world, join=True)
    full = finish_stats(torch.stack([record(b) for b in batches()])).numpy()
    for r in range(world):
        red = ret[r]
        assert np.array_equal(red[:, [H.ST_MIN, H.ST_MAX, H.ST_NAN, H.ST_N]],
                              full[:, [H.ST_MIN, H.ST_MAX, H.ST_NAN, H.ST_N]])
        np.testing.assert_allclose(red[:, H.ST_MEANABS], full[:, H.ST_MEANABS], rtol=1e-6, equal_nan=True)
        np.testing.assert_allclose(red[:, H.ST_STD], full[:, H.ST_STD], rtol=1e-6, equal_nan=True)
    # running-state replay equals the reference's sequential observer on the full batches
    mn, mx = 0, 0
    for b in batches():
        mn, mx = O.observe_minmax(b, mn, mx)
    rmn, rmx = replay_minmax(0, 0, ret[0][:, [H.ST_MIN, H.ST_MAX, H.ST_NAN]].tolist())
    assert (rmn, rmx) == (mn, mx)
    assert O.minmax_qparams(rmn, rmx, False) == O.minmax_qparams(mn, mx, False)
    # the NaN call contributes nothing, its fp32 means are NaN like torch's
    assert np.isnan(ret[0][2, H.ST_MEANABS])


def test_replay_minmax_tensor_equals_sequential_fold():
    """The vectorized replay (bench C5 / large calibrations) equals the reference fold."""
    import numpy as np
    import torch
    from vsiquantization_amd import _hip as H
    from vsiquantization_amd.distributed import replay_minmax, replay_minmax_tensor
    rng = np.random.default_rng(0)
    recs = torch.zeros(5, 7, H.ST_LEN, dtype=torch.float64)
    recs[..., H.ST_MIN] = torch.from_numpy(rng.normal(size=(5, 7)))
    recs[..., H.ST_MAX] = torch.from_numpy(rng.normal(size=(5, 7)) + 1)
    recs[1, 3, H.ST_NAN] = 2                       # a NaN call is skipped
    recs[2, :, H.ST_MIN] = 0.5                     # never below the initial 0
    recs[3, :, H.ST_MIN] = -0.0                    # -0.0 does not replace 0 (strict <)
    init = [(0, 0), (-3.0, 0.5), (0, 0), (0, 0), (1.0, 1.0)]
    mn, mx = replay_minmax_tensor([a for a, _ in init], [b for _, b in init], recs)
    for i, (a, b) in enumerate(init):
        calls = recs[i][:, [H.ST_MIN, H.ST_MAX, H.ST_NAN]].tolist()
        want = replay_minmax(a, b, calls)
        got = (float(mn[i]), float(mx[i]))
        assert got == tuple(float(w) for w in want)
        assert np.signbit(got[0]) == np.signbit(float(want[0]))


def _count_worker(rank, world, port, counts_by_rank, ret):
    from vsiquantization_amd.distributed import check_call_counts
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        check_call_counts(counts_by_rank[rank], torch.device("cpu"))
        ret[rank] = "ok"
    except RuntimeError as e:
        ret[rank] = str(e)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("counts,ok", [([[16, 16, 16], [16, 16, 16]], True),
                                       ([[16, 16, 16], [16, 16, 15]], False),    # one missing call
                                       ([[16, 16, 16], [16, 16]], False),        # one missing layer
                                       ([[16, 15, 16], [15, 16, 16]], False)])   # same total, moved
def test_sync_calibration_call_count_check(counts, ok):
    """sync_calibration's pre-check (distributed.check_call_counts): every rank raises the
    same error when the ranks' deferred calls differ, instead of folding different calls
    together (uneven shards)."""
    port = 29600 + os.getpid() % 1000
    ret = mp.Manager().dict()
    mp.spawn(_count_worker, args=(2, port, counts, ret), nprocs=2, join=True)
    if ok:
        assert ret[0] == ret[1] == "ok"
    else:
        assert "different deferred observer calls" in ret[0] and "different deferred observer calls" in ret[1]


def _gather_worker(rank, world, port, ret):
    from vsiquantization_amd.distributed import gather_stats
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        st = torch.arange(H.ST_LEN, dtype=torch.float64) + 100 * rank
        ret[rank] = gather_stats(st).numpy().copy()
    finally:
        dist.destroy_process_group()


def test_gather_stats_rank_order():
    """distributed.gather_stats (the per-call exchange: ONE collective per observer call,
    folded on the device by vsiq_observe_finalize_ranks): every rank holds all records in
    rank order."""
    port = 29700 + os.getpid() % 1000
    ret = mp.Manager().dict()
    mp.spawn(_gather_worker, args=(3, port, ret), nprocs=3, join=True)
    want = np.concatenate([np.arange(H.ST_LEN) + 100 * r for r in range(3)]).astype(np.float64)
    for r in range(3):
        assert np.array_equal(ret[r], want)
