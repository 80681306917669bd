"""Whole-step HIP-graph capture for QAT steps built on this package (MI355X-native
replacement for a tracing compiler: the reference runs every step eagerly, one Python
dispatch per op).

Every kernel of the package launches on torch's current stream, never synchronises the
host and keeps its reduction workspace per capture (`_hip.workspace`), so a forward +
backward through the public API (FakeQuantize / QuantizationManager / the fused layers,
quantizers/uniform.py:34-56, observers/minmax.py:32-88) can be captured once and
replayed: the replay costs the GPU time plus one graph launch, whatever the number of
layers.  ``GraphedStep`` adds the two things a capture of this package needs: warm-up
steps on a side stream (allocator pools, lazily created tensors), and, before the
capture, steps until the store-gate tuner has settled every launch site the step uses
(a capture bakes the gate in; csrc/gate_tune.hip never times a captured launch).

    step = GraphedStep(lambda: model(x).square().mean().backward(), grads_of=model.parameters())
    for _ in range(iters):
        step()            # replay; inputs are updated in place (x.copy_(batch))
"""
from __future__ import annotations

import torch

from .. import _hip as H


def quiesce_collectives(groups=None) -> None:
    """Call right before a HIP-graph capture: finishes the device's work and, under RCCL,
    makes sure every group this package's collectives use has its capture-only twin
    (vsiquantization_amd.distributed.prepare_capture; collective: every rank calls it).
    The collectives captured next run on the twins, which never run an eager collective,
    so no eager and captured RCCL work meet on one communicator (no timed wait: round 5's
    0.3 s settle for ProcessGroupNCCL's watchdog is gone)."""
    torch.cuda.synchronize()
    from .. import distributed as D
    D.prepare_capture(groups)


def _detached(v):
    if isinstance(v, torch.Tensor):
        return v.detach()
    if isinstance(v, (list, tuple)):
        return type(v)(_detached(u) for u in v)
    if isinstance(v, dict):
        return {k: _detached(u) for k, u in v.items()}
    return v


class GraphedStep:
    """Capture ``fn`` (no arguments; reads and writes persistent tensors) into a HIP graph.

    ``fn`` runs ``warmup`` times on a side stream, then until the store-gate tuner has no
    site left to tune (at most ``settle_max`` more runs), then once under capture.  Under
    torch.distributed (``group``, default the world when initialised) the ranks agree on
    that stop -- MAX of their pending counts each run -- so a step holding a collective
    (DDP's all-reduce) runs equally often on every rank.  Calling
    the object replays the graph on the current stream and returns what the captured run
    returned (its tensors are overwritten by every replay).  ``grads_of``: tensors whose
    ``.grad`` is set to None before each warm-up run and before the capture, so that the
    captured backward WRITES their gradients (AccumulateGrad then keeps the produced
    buffer) and every replay leaves exactly one step's gradient there.
    """

    def __init__(self, fn, warmup: int = 3, settle_max: int = 400, grads_of=(), group=None):
        self.fn = fn
        self.params = list(grads_of)
        self.group = group
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._clear()
                fn()
            torch.cuda.current_stream().synchronize()
            H.gate_tuning_pending()   # from here on: the sites this step launches
            for _ in range(settle_max):
                self._clear()
                fn()
                torch.cuda.current_stream().synchronize()
                if self._pending() == 0:
                    break
        torch.cuda.current_stream().wait_stream(side)
        self._clear()
        quiesce_collectives()
        self.graph = torch.cuda.CUDAGraph()
        before = set(H._WS)
        # thread_local: other threads of the process (torch's NCCL watchdog polling the events
        # of earlier collectives, autograd's device threads) may keep calling the runtime
        # while this thread captures; "global" mode turns those calls into capture errors
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self._cids = [H._capture_id(H.stream_of(torch.cuda.current_device()))]
            out = fn()
        # keep the outputs' storage (every replay rewrites it), not their autograd graph:
        # a live graph would keep the parameters' AccumulateGrad nodes of the capture
        # stream alive into later eager steps (torch's stream-mismatch warning)
        self.out = _detached(out)
        del out
        # the capture's own reduction workspaces / counters (one per capture, from the
        # graph's pool): released with this object, not kept by _hip's table forever
        self._ws_keys = [k for k in H._WS if k not in before]

    def _pending(self) -> int:
        n = H.gate_tuning_pending()
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return n
        g = self.group if self.group is not None else dist.group.WORLD
        if dist.get_world_size(g) == 1:
            return n
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(g) == "nccl" else "cpu"
        t = torch.tensor([n], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g)
        return int(t)

    def _clear(self):
        for p in self.params:
            p.grad = None

    def __call__(self):
        self.graph.replay()
        return self.out

    def _drop_workspaces(self):
        for k in getattr(self, "_ws_keys", ()):
            H._WS.pop(k, None)
        self._ws_keys = []
        cids = [c for c in getattr(self, "_cids", ()) if c is not None]
        self._cids = []
        if cids and H._EXT is not None:   # the C++ nodes' capture workspaces
            H._EXT.release_captures(cids)

    def release(self):
        """Drop the graph and the workspaces its capture allocated."""
        self._drop_workspaces()
        self.graph = None
        self.out = None

    def __del__(self):
        try:
            self._drop_workspaces()
        except Exception:   # interpreter shutdown
            pass
