"""HIP-graph capture of the learnable fake-quant step (MI355X-native replacement for a
tracing compiler): the kernels take torch's current stream and never sync the host, so
a fwd + bwd through the public API (quantizers/uniform.py:34-56 -> K1 / K4) can be
captured with torch.cuda.graph and replayed; replays give the eager results bit for bit.
"""
import pytest
import torch

import vsiquantization_amd as V

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _step(q, x, g, s, act):
    y = q.quantize(x, s, 0, True, act=act)
    y.backward(g)
    return y


@pytest.mark.parametrize("act", [None, "relu"])
def test_learnable_step_graph_replay_equals_eager(act):
    torch.manual_seed(0)
    q = V.UniformQuantizer(4, True)
    x = torch.randn(3, 16, 40, 40, device=DEV, requires_grad=True)
    g = torch.randn(3, 16, 40, 40, device=DEV)
    s = torch.nn.Parameter(torch.tensor(0.07, dtype=torch.float64, device=DEV))

    y_ref = _step(q, x, g, s, act).detach().clone()
    gx_ref, gs_ref = x.grad.clone(), s.grad.clone()

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):          # warm up on the capture-side stream
        for _ in range(2):
            x.grad, s.grad = None, None
            _step(q, x, g, s, act)
    torch.cuda.current_stream().wait_stream(side)

    x.grad, s.grad = None, None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        y = _step(q, x, g, s, act)
    for _ in range(3):
        x.grad.zero_()
        s.grad.zero_()
        graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)
    assert torch.equal(x.grad, gx_ref)
    assert torch.equal(s.grad, gs_ref)
