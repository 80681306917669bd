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


def test_fused_model_training_step_graph_replay_equals_eager():
    """A fused ConvBnReLU model after calibration + activate_learning_qparam +
    activate_quantizer (modules/fused.py, utils/quantize_manager.py): forward, loss and
    backward captured in one graph (MIOpen convs and the fake-quant kernels together);
    replay == eager bit for bit for the output, the conv biases and the activation
    quantizers' f64 scale gradients; conv weights and weight-quantizer scales within
    1e-5 (MIOpen's weight-gradient convolution is not bit-reproducible run to run)."""
    import torch.nn as nn
    from vsiquantization_amd.modules.fused import ConvBnReLU
    from vsiquantization_amd.utils.quantize_manager import (activate_learning_qparam, activate_quantizer,
                                                            calibrate_qat_model, data_calib)
    torch.manual_seed(0)
    layers = []
    for cin, cout in ((3, 8), (8, 16)):
        bn = nn.BatchNorm2d(cout)
        bn.running_var.uniform_(0.5, 2.0)
        layers.append(ConvBnReLU(nn.Conv2d(cin, cout, 3, padding=1, bias=False), bn, nn.ReLU(),
                                 "MinMaxObserver", "UniformQuantizer", "MinMaxObserver", "UniformQuantizer",
                                 True, True, True, 4, 4))
    model = nn.Sequential(*layers).to(DEV)
    gen = torch.Generator().manual_seed(1)
    loader = [(torch.randint(0, 256, (2, 3, 16, 16), generator=gen, dtype=torch.uint8), None) for _ in range(2)]
    calibrate_qat_model(model, loader, data_calib, DEV)
    activate_learning_qparam(model)
    activate_quantizer(model)
    model.eval()   # BN folded; eval keeps the step free of running-stat updates
    x = torch.rand(2, 3, 16, 16, device=DEV)
    named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
    params = [p for _, p in named]
    # the learnable f64 scales are created where the layer's tensors live (no model.to())
    assert all(p.device.type == "cuda" for p in params)
    assert model[0].activation_quantizer.scale.dtype == torch.float64

    def step():
        out = model(x)
        out.square().mean().backward()
        return out

    for p in params:
        p.grad = None
    out_ref = step().detach().clone()
    grads_ref = [p.grad.clone() for p in params]

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            for p in params:
                p.grad = None
            step()
    torch.cuda.current_stream().wait_stream(side)
    for p in params:
        p.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = step()
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, out_ref)
    for (name, p), gr in zip(named, grads_ref):
        if name.endswith("conv_fuse.weight") or name.endswith("weight_quantizer.scale"):
            # MIOpen's weight-gradient convolution is not bit-reproducible between the eager
            # and the captured run (~1e-7 relative); the weight quantizer's scale gradient
            # is computed by K7/K4 from that incoming gradient
            torch.testing.assert_close(p.grad, gr, rtol=1e-5, atol=1e-12, msg=name)
        else:
            assert torch.equal(p.grad, gr), name


def test_two_graphs_own_workspaces_and_replay_concurrently():
    """Each captured graph gets its own reduction workspace + arrival counter (keyed by
    the capture id: _hip.workspace, or the C++ nodes' cache in _vsiq_torch.so), so two graphs replayed at the same time on two
    streams do not share a counter: both give their eager results bit for bit."""
    from vsiquantization_amd import _hip as H
    torch.manual_seed(1)
    q = V.UniformQuantizer(8, True)
    xs = [torch.randn(64, 32, 56, 56, device=DEV, requires_grad=True) for _ in range(2)]
    gs = [torch.randn(64, 32, 56, 56, device=DEV) for _ in range(2)]
    ss = [torch.nn.Parameter(torch.tensor(v, dtype=torch.float64, device=DEV)) for v in (0.03, 0.05)]
    ref = []
    for x, g, s in zip(xs, gs, ss):
        _step(q, x, g, s, None)
        ref.append((x.grad.clone(), s.grad.clone()))
        x.grad, s.grad = None, None
    # the learnable C++ node keeps its workspaces in the extension, the Python path in _hip
    ext = H.torch_ext() if H.torch_ext_enabled() else None
    before = {k for k in H._WS if "capture" in k}
    before_c = ext.capture_workspaces() if ext else 0
    graphs = []
    for x, g, s in zip(xs, gs, ss):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            _step(q, x, g, s, None)
        torch.cuda.current_stream().wait_stream(side)
        x.grad, s.grad = None, None
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            _step(q, x, g, s, None)
        graphs.append(gr)
    new = {k for k in H._WS if "capture" in k} - before
    new_c = (ext.capture_workspaces() - before_c) if ext else 0
    assert len(new) + new_c == 2, (new, new_c)
    streams = [torch.cuda.Stream() for _ in range(2)]
    for _ in range(5):
        for x, s in zip(xs, ss):
            x.grad.zero_()
            s.grad.zero_()
        torch.cuda.synchronize()
        for gr, st in zip(graphs, streams):
            with torch.cuda.stream(st):
                gr.replay()
        torch.cuda.synchronize()
        for (gx, gsr), x, s in zip(ref, xs, ss):
            assert torch.equal(x.grad, gx)
            assert torch.equal(s.grad, gsr)


def test_graphed_step_c2_public_api_equals_eager():
    """utils.graph.GraphedStep on the C2 step through the public API
    (PerChannelMinMaxObserver.observe_quantize + backward): every replay gives the eager
    y and dW bit for bit (fresh observer state each step: the same weight, so the same
    running min/max), and the tuner had settled before the capture."""
    from vsiquantization_amd import _hip as H
    from vsiquantization_amd.utils.graph import GraphedStep
    torch.manual_seed(3)
    w = (torch.randn(1024, 256, 3, 3, device=DEV) * 0.05).requires_grad_(True)
    g = torch.randn_like(w)
    obs, q = V.PerChannelMinMaxObserver(False), V.PerChannelUniformQuantizer(8, False)

    def step():
        y, _ = obs.observe_quantize(w, q)
        y.backward(g)
        return y

    w.grad = None
    y_ref = step().detach().clone()
    gw_ref = w.grad.clone()
    gs = GraphedStep(step, grads_of=[w])
    torch.cuda.synchronize()
    H.gate_tuning_pending()
    step()          # an eager step launches the same sites: all of them settled
    torch.cuda.synchronize()
    assert H.gate_tuning_pending() == 0
    w.grad = None
    gs = GraphedStep(step, grads_of=[w])
    for _ in range(3):
        y = gs()
    torch.cuda.synchronize()
    assert torch.equal(y.view(torch.int32), y_ref.view(torch.int32))
    assert torch.equal(w.grad.view(torch.int32), gw_ref.view(torch.int32))
