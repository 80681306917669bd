"""Multi-GPU observer: batch-sharded activations, one process per GPU (RCCL over xGMI).

The fake-quant itself is elementwise and needs no communication.  The only
exchange is the per-tensor observer's statistics: every rank
runs the observer pass over its shard and writes its stats record(s); ONE
all_gather of the records (``all_gather_into_tensor`` on every backend), then a
fold in rank order on every rank -- min / max exact, the sums in float64 in a fixed
order, so every rank holds the same bits -- followed by the reference's running
update (observers/minmax.py:42-47) and the f64 qparams.  min/max and the qparams are
bit-identical to a 1-GPU run (no activation or ReLU; a fused SiLU follows each rank's
own shard layout, as F.silu does under the reference's DDP: pinned per shard against the
oracle, and against a whole-batch run it differs only where the two layouts pick a
different exp path -- tests/test_gpu_dist_calib.py::test_sharded_silu_follows_each_ranks_layout);
the sums differ only in float64 summation order.
(``allreduce_stats`` -- MAX over [-min, max], SUM over the sums -- is what the
deferred sync uses over all records of all layers at once.)

Two modes:
* per call  (``QuantizationManager.dist_group`` set, ``dist_defer`` False): one tiny
  all_gather of the stats records per observer call; an observe+quantize call (§3.4)
  then folds them inside its fake-quant launch (``observe_gather_fake_quant``: two
  launches and one collective per call), an observe-only call in one fold launch
  (``gather_finalize``);
* deferred  (``dist_defer`` True, calibration): each rank only writes its local
  per-call partial records (K2p, no cross-workgroup fold, no atomics);
  ``sync_calibration(model)`` folds ALL calls of ALL layers in one launch,
  all-reduces the records in two collectives and replays the running min/max per
  layer.  With ``dist_group`` None it is a single-GPU deferred calibration (no
  collective).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _hip as H

_SUM_SLICE = slice(H.ST_NAN, H.ST_N + 1)

# ---------------------------------------------------------------- HIP-graph capture groups
# A collective of this package issued inside a HIP-graph capture on RCCL runs on a
# capture-only TWIN of its process group (prepare_capture): a communicator that never
# runs an eager collective.  So, by construction, (1) no eager and captured RCCL
# operations are ever mixed on one communicator, (2) the eager group's NCCL stream never
# joins a capture, and (3) the twin's ProcessGroupNCCL watchdog never holds a work to
# poll (captured collectives are never listed and graph replays list nothing) -- the
# three ways a capture could meet the watchdog or RCCL's eager state (round 5 saw one
# watchdog SIGABRT inside such a capture; tools/exp/rccl_capture_probe.py shows polling a
# listed work's event during a capture does not fail by itself on this ROCm).
_TWINS = {}   # id(group) -> (group, its capture-only twin)
_USED = {}    # id(group) -> group: groups this package's collectives ran on, first-use order


def _world(group):
    return group if group is not None else dist.group.WORLD


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _resolve(group):
    """The process group a collective of this package runs on: `group`, or under a
    HIP-graph capture on RCCL its capture-only twin (prepare_capture must have created it:
    groups cannot be created inside a capture)."""
    g = _world(group)
    _USED.setdefault(id(g), g)
    if _capturing() and dist.get_backend(g) == "nccl":
        tw = _TWINS.get(id(g))
        if tw is None:
            raise RuntimeError("an RCCL collective of vsiquantization_amd inside a HIP-graph capture needs the "
                               "group's capture-only twin: call vsiquantization_amd.distributed.prepare_capture() "
                               "on every rank before capturing (GraphedStep and bench.capture_groups do)")
        return tw[1]
    return group


collective_group = _resolve   # public name: the group to pass to a collective issued by hand


def capture_group(group=None):
    """The capture-only twin of `group` (None: the world) after prepare_capture, else None."""
    tw = _TWINS.get(id(_world(group)))
    return tw[1] if tw else None


def prepare_capture(groups=None) -> int:
    """Create (collectively: every rank calls it, with the same groups) the capture-only
    RCCL twin of every group this package's collectives have used so far -- or of
    `groups` -- plus the world, eagerly initialised on the current device.  Idempotent;
    nothing to do without an NCCL process group.  Returns the number of twins."""
    if not (dist.is_available() and dist.is_initialized()):
        return 0
    gs = [_world(g) for g in groups] if groups is not None else list(_USED.values())
    gs.append(dist.group.WORLD)
    uniq = {}
    for g in gs:
        uniq.setdefault(id(g), g)
    # the same creation order on every rank: by member ranks (first use breaks ties)
    order = [g for g in sorted(uniq.values(), key=lambda g: tuple(dist.get_process_group_ranks(g)))
             if id(g) not in _TWINS and dist.get_backend(g) == "nccl"]
    if order:
        dev = torch.device("cuda", torch.cuda.current_device())
    for g in order:
        twin = dist.new_group(dist.get_process_group_ranks(g), backend="nccl", device_id=dev)
        _TWINS[id(g)] = (g, twin)
    return len(_TWINS)


def release_capture_groups():
    """Destroy the capture-only twins (e.g. before destroy_process_group of their groups)."""
    for g, twin in list(_TWINS.values()):
        try:
            dist.destroy_process_group(twin)
        except Exception:  # noqa: BLE001  (already torn down with the world)
            pass
    _TWINS.clear()


def finish_stats(stats: torch.Tensor) -> torch.Tensor:
    """Recompute the fp32-rounded mean|x|, mean, std entries from the sums (in place)."""
    n = stats[..., H.ST_N]
    mean = stats[..., H.ST_SUM] / n
    var = (stats[..., H.ST_SUMSQ] - stats[..., H.ST_SUM] * mean) / (n - 1.0)
    has_nan = stats[..., H.ST_NAN] > 0
    nan = torch.full_like(mean, float("nan"))
    std = torch.where(n > 1, var.clamp_min(0.0).sqrt(), nan)
    vals = [stats[..., H.ST_SUMABS] / n, mean, std]
    for i, v in zip((H.ST_MEANABS, H.ST_MEAN, H.ST_STD), vals):
        stats[..., i] = torch.where(has_nan, nan, v.to(torch.float32).to(torch.float64))
    return stats


def allreduce_stats(stats: torch.Tensor, group=None) -> torch.Tensor:
    """All-reduce observer stats records ``[..., ST_LEN]`` across ranks, in place."""
    mm = torch.stack([-stats[..., H.ST_MIN], stats[..., H.ST_MAX]], dim=-1).contiguous()
    sums = stats[..., _SUM_SLICE].contiguous()
    group = _resolve(group)
    dist.all_reduce(mm, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
    stats[..., H.ST_MIN] = -mm[..., 0]
    stats[..., H.ST_MAX] = mm[..., 1]
    stats[..., _SUM_SLICE] = sums
    return finish_stats(stats)


def gather_stats(stats: torch.Tensor, group=None, out: torch.Tensor | None = None) -> torch.Tensor:
    """One collective: every rank's stats record ``[ST_LEN]`` gathered in rank order into
    ``[world * ST_LEN]`` (all_gather_into_tensor, on RCCL and on the gloo rehearsals
    alike, so the tests run the branch the multi-GPU job runs)."""
    world = dist.get_world_size(group)
    if out is None:
        out = torch.empty(world * H.ST_LEN, dtype=stats.dtype, device=stats.device)
    dist.all_gather_into_tensor(out, stats.contiguous(), group=_resolve(group))
    return out


def gather_finalize(stats: torch.Tensor, run_minmax: torch.Tensor, *, symmetric: bool, num_bits: int = 8,
                    eps: float = 1e-8, group=None):
    """Per-call multi-GPU observer exchange (observe only): gather the ranks' stats records
    (one collective), then ONE launch folds them in rank order (min / max exact, sums in
    float64 -- the same bits on every rank), writes the batch's stats record and applies
    the running update + f64 qparams (vsiq_observe_finalize_ranks).  Returns (stats
    f64[ST_LEN], qp f64[QP_LEN]); min/max/qparams bit-identical to one GPU over the whole
    batch when the ranks' records were taken with act None / "relu" (a fused SiLU follows
    each rank's own shard layout; see observe_gather_fake_quant)."""
    from .fakequant import qden
    gathered = gather_stats(stats, group)
    dev = stats.device
    st = torch.empty(H.ST_LEN, dtype=torch.float64, device=dev)
    qp = torch.empty(H.QP_LEN, dtype=torch.float64, device=dev)
    rc = H.lib().vsiq_observe_finalize_ranks(H.ptr(gathered), int(dist.get_world_size(group)), H.ptr(st),
                                             H.ptr(run_minmax), H.ptr(qp), int(bool(symmetric)),
                                             qden(symmetric, num_bits, eps), float(eps), H.stream_of(dev))
    H.check(rc, "vsiq_observe_finalize_ranks")
    return st, qp


def observe_gather_fake_quant(x: torch.Tensor, run_minmax: torch.Tensor, *, symmetric: bool, num_bits: int = 8,
                              eps: float = 1e-8, qmin: int, qmax: int, act=None, group=None,
                              want_mask: bool = False):
    """Per-call multi-GPU observe + fake quant of this rank's shard (observe+quantize mode,
    quantization_manager.py:73-90 under DDP): the local K2 pass (stats record only), ONE
    all_gather of the ranks' records, and ONE launch that folds them in rank order, applies
    the running update + f64 qparams and fake-quantizes act(x) (vsiq_act_fq_fwd_ranks_f32).
    Two launches and one collective per call; for act None / "relu", min / max / qparams / y
    are bit-identical to one GPU over the whole batch.  A fused SiLU follows the reference
    CPU layout of THIS RANK's shard (its own size and local element indices decide which
    elements take glibc's scalar exp), so SiLU parity with a 1-GPU run over the whole batch
    is not pinned -- each rank equals the reference's F.silu on its own shard.
    Returns (y, qp f64[QP_LEN], stats f64[ST_LEN], mask | None)."""
    from .fakequant import _i64, observe_tensor, qden
    x = H.require_device_f32(x)
    _, local = observe_tensor(x, symmetric=symmetric, num_bits=num_bits, eps=eps, run_minmax=None,
                              want_qp=False, want_stats=True, act=act)
    gathered = gather_stats(local, group)
    dev = x.device
    y = torch.empty_like(x)
    qp = torch.empty(H.QP_LEN, dtype=torch.float64, device=dev)
    st = torch.empty(H.ST_LEN, dtype=torch.float64, device=dev)
    mask = H.mask_buffer(1, x.numel(), dev) if want_mask else None
    rc = H.lib().vsiq_act_fq_fwd_ranks_f32(H.ptr(x), H.ptr(y), None, H.ptr(mask), _i64(x.numel()), H.act_code(act),
                                           H.ptr(gathered), int(dist.get_world_size(group)), H.ptr(st),
                                           H.ptr(run_minmax), H.ptr(qp), int(bool(symmetric)),
                                           qden(symmetric, num_bits, eps), float(eps), int(qmin), int(qmax),
                                           H.stream_of(dev))
    H.check(rc, "vsiq_act_fq_fwd_ranks_f32")
    return y, qp, st, mask


class ObserveGatherFakeQuantFn(torch.autograd.Function):
    """observe_gather_fake_quant with the reference's STE gradient at fp32(scale) of this
    call (FakeQuantFixedFn's backward; x only)."""

    @staticmethod
    def forward(ctx, x, run_minmax, symmetric, num_bits, eps, qmin, qmax, act, group):
        y, qp, st, mask = observe_gather_fake_quant(x, run_minmax, symmetric=symmetric, num_bits=num_bits, eps=eps,
                                                    qmin=qmin, qmax=qmax, act=act, group=group, want_mask=True)
        ctx.act = act
        ctx.save_for_backward(mask, x) if H.act_code(act) != H.ACT_NONE else ctx.save_for_backward(mask)
        ctx.scale = qp[H.QP_SCALE:H.QP_SCALE + 1]
        ctx.mark_non_differentiable(qp, st)
        return y, qp, st

    @staticmethod
    def backward(ctx, gy, _gqp, _gst):
        from .fakequant import ste_backward
        saved = ctx.saved_tensors
        pre = saved[1] if len(saved) > 1 else None
        gx = ste_backward(gy.contiguous(), saved[0], ctx.scale, pre=pre, act=ctx.act)
        return gx, None, None, None, None, None, None, None, None


def replay_minmax(min_val, max_val, records):
    """Fold per-call [min, max, nan_count] records into the running state exactly like
    observers/minmax.py:42-47 (a NaN call changes nothing; strict comparisons)."""
    for mn, mx, nanc in records:
        if nanc > 0:
            continue
        if mn < min_val:
            min_val = mn
        if mx > max_val:
            max_val = mx
    return min_val, max_val


def replay_minmax_tensor(init_min, init_max, recs: torch.Tensor):
    """Vectorized replay_minmax over a batch of layers: recs [layers, calls, ST_LEN] (any
    device), init_min/init_max [layers] -> (min [layers], max [layers]) f64 tensors.

    Equal to the sequential fold: under strict comparisons the running minimum ends as
    the smallest call minimum when that is strictly below the initial value (equal
    values are the same bits except +-0, which a strict compare never swaps), else the
    initial value; NaN calls are skipped."""
    nan_call = recs[..., H.ST_NAN] > 0
    mins = recs[..., H.ST_MIN].masked_fill(nan_call, float("inf")).amin(dim=-1)
    maxs = recs[..., H.ST_MAX].masked_fill(nan_call, float("-inf")).amax(dim=-1)

    def as_t(v):   # python numbers stay host scalars (no host->device copy, no sync)
        if isinstance(v, torch.Tensor):
            return v.to(recs.device, recs.dtype)
        if isinstance(v, (list, tuple)):
            return torch.tensor(v, dtype=recs.dtype).to(recs.device, non_blocking=True)
        return torch.full_like(mins, float(v))

    lo, hi = as_t(init_min), as_t(init_max)
    return torch.where(mins < lo, mins, lo), torch.where(maxs > hi, maxs, hi)


def check_call_counts(counts, device, group=None):
    """All ranks must hold the same deferred calls (managers x calls each) before their
    records are all-reduced row by row: a rank with an extra or missing calibration batch
    would otherwise fold different calls together (or hang on mismatched sizes).  One
    tiny MAX all-reduce of [h, -h] over (manager count, call count, order hash); raises
    RuntimeError on every rank when any differs."""
    h = 0
    for c in counts:
        h = (h * 1000003 + int(c) + 1) % 2147483647
    head = torch.tensor([len(counts), sum(counts), h], dtype=torch.float64)
    both = torch.cat([head, -head]).to(device)
    dist.all_reduce(both, op=dist.ReduceOp.MAX, group=_resolve(group))
    hi, lo = both[:3].cpu(), -both[3:].cpu()
    if not torch.equal(hi, lo):
        raise RuntimeError(f"sync_calibration: ranks hold different deferred observer calls "
                           f"(managers / calls: local {len(counts)} / {sum(counts)}, across ranks "
                           f"{int(lo[0])}..{int(hi[0])} / {int(lo[1])}..{int(hi[1])}); every rank "
                           "must run the same calibration batches through the same layers")


def fold_slots(slots):
    """Stats records [calls, ST_LEN] of K2p slots of any sizes, in call order: one
    fold_parts launch per distinct slot length (each call's slot is sized for its
    tensor, part_slot_doubles(numel), instead of the largest possible)."""
    from .fakequant import fold_parts
    by_len = {}
    for i, p in enumerate(slots):
        by_len.setdefault(p.numel(), []).append(i)
    if len(by_len) == 1:
        return fold_parts(torch.stack(slots))
    order, parts = [], []
    for idx in by_len.values():
        order.extend(idx)
        parts.append(fold_parts(torch.stack([slots[i] for i in idx])))
    inv = torch.empty(len(order), dtype=torch.int64)
    inv[torch.tensor(order)] = torch.arange(len(order))
    return torch.cat(parts).index_select(0, inv.to(slots[0].device, non_blocking=True))


def _deferred_managers(model):
    from .quantizers.quantization_manager import QuantizationManager
    for m in model.modules():
        if isinstance(m, QuantizationManager) and m._pending_records:
            yield m


def sync_calibration(model, group=None):
    """Deferred calibration sync: ONE fold launch over every recorded call of every layer
    (K2p slots -> stats records), then -- across ranks -- two all-reduces, then the exact
    running-state replay per layer.  ``group``: the process group of the all-reduce;
    None = the managers' own ``dist_group`` (no collective when that is None too: a
    single-GPU deferred calibration)."""
    mgrs = list(_deferred_managers(model))
    if not mgrs:
        return 0
    from . import observe_batch
    observe_batch.flush()   # queued deferred calls (K2m) write their records now
    for m in mgrs:
        m._join()   # records may still be in flight on an observer side stream
    counts = [len(m._pending_records) for m in mgrs]
    if group is None:
        groups = {id(m.dist_group): m.dist_group for m in mgrs if m.dist_group is not None}
        if len(groups) > 1:
            raise RuntimeError("sync_calibration: managers use different dist_group values; "
                               "pass group= explicitly")
        group = next(iter(groups.values()), None)
        collective = group is not None
    else:
        collective = True
    slots = [p for m in mgrs for p in m._pending_records]
    dev = slots[0].device
    if collective:
        check_call_counts(counts, dev, group)
    stats = fold_slots(slots)
    if collective:
        stats = allreduce_stats(stats, group=group)
    host = stats.cpu()
    for m, part in zip(mgrs, host.split(counts)):
        m._apply_synced_records(part)
    return len(mgrs)
