"""The C++ autograd nodes of _vsiq_torch.so (csrc/torch_ops.cpp) against the Python
autograd.Functions over ctypes (VSIQ_TORCH_EXT=0): same kernels, so every output and
gradient must be bit-identical.  The rest of the -m gpu suite runs the public API on the
C++ nodes (the default) against the oracle and the reference goldens."""
import numpy as np
import pytest
import torch

import vsiquantization_amd as V
from vsiquantization_amd import _hip as H
from vsiquantization_amd.quantizers.lsq_module import LSQFakeQuantize

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _bits(t):
    """bit pattern (NaN-safe equality)"""
    t = t.detach().cpu().contiguous()
    return t.view({torch.float32: torch.int32, torch.float64: torch.int64}.get(t.dtype, t.dtype))


def both(fn, monkeypatch):
    """fn() under the C++ nodes, then under the Python Functions."""
    out = []
    for ext in (True, False):
        monkeypatch.setattr(H, "torch_ext_enabled", lambda e=ext: e)
        out.append(fn())
    monkeypatch.undo()
    return out


def test_extension_loads():
    ext = H.torch_ext()
    assert ext.abi_version() == H.ABI_VERSION


@pytest.mark.parametrize("shape,sym", [((64, 32, 3, 3), False), ((48, 27), True), ((5, 1000), False),
                                       ((1024, 1024, 3, 3), False)])
def test_pc_observe_quantize_ext_equals_python(shape, sym, monkeypatch):
    g0 = torch.Generator(device=DEV).manual_seed(1)
    w = torch.randn(shape, device=DEV, generator=g0) * 0.05
    w[1, 0] = float("nan") if shape[0] > 2 else w[1, 0]
    g = torch.randn(shape, device=DEV, generator=g0)

    def run():
        x = w.clone().requires_grad_(True)
        obs = V.PerChannelMinMaxObserver(sym)
        y, rs = obs.observe_quantize(x, V.PerChannelUniformQuantizer(8, sym), want_row_stats=True)
        y.backward(g)
        return y, x.grad, obs.scale, obs.zero_point, rs, obs.run_min, obs.run_max

    a, b = both(run, monkeypatch)
    for u, v in zip(a, b):
        assert torch.equal(_bits(u), _bits(v))


def test_pc_observe_quantize_bound_op_and_its_fallbacks(monkeypatch):
    """The public-API step's bound C++ op (PcObserveFqOp: its own eligibility checks, one
    allocation for scale / zp / mask): a sequence of calls that takes it, then calls it
    must hand back (no grad mode, x without grad, a non-contiguous x, another row count),
    gives the same y / grad / scale / zp / running state bits as the Python Functions,
    and every call's scale / zp are new tensors (an earlier call's values stay as they were)."""
    g0 = torch.Generator(device=DEV).manual_seed(3)
    ws = [torch.randn(64, 16, 3, 3, device=DEV, generator=g0) * s for s in (0.05, 0.2, 0.01)]
    w_other = torch.randn(32, 16, 3, 3, device=DEV, generator=g0) * 0.1
    g = torch.randn(64, 16, 3, 3, device=DEV, generator=g0)

    def run():
        obs, q = V.PerChannelMinMaxObserver(False), V.PerChannelUniformQuantizer(8, False)
        out, kept = [], []
        for i, w in enumerate(ws * 2):
            x = w.clone().requires_grad_(True)
            y, _ = obs.observe_quantize(x, q)
            y.backward(g)
            out += [y, x.grad, obs.scale, obs.zero_point, obs.run_min, obs.run_max]
            kept.append((obs.scale, obs.scale.clone(), obs.zero_point, obs.zero_point.clone()))
        with torch.no_grad():
            out += list(obs.observe_quantize(ws[0].clone().requires_grad_(True), q)[:1])
        out += list(obs.observe_quantize(ws[1], q)[:1])
        xt = ws[2].transpose(2, 3).requires_grad_(True)    # non-contiguous
        y, _ = obs.observe_quantize(xt, q)
        y.backward(g)
        out += [y, xt.grad, obs.scale]
        xo = w_other.clone().requires_grad_(True)   # another row count: the state restarts
        y, _ = obs.observe_quantize(xo, q)
        out += [y, obs.scale, obs.run_min]
        for s, s0, z, z0 in kept:
            assert torch.equal(_bits(s), _bits(s0)) and torch.equal(_bits(z), _bits(z0))
        return out

    a, b = both(run, monkeypatch)
    assert len(a) == len(b)
    for u, v in zip(a, b):
        assert u.shape == v.shape and torch.equal(_bits(u), _bits(v))


def test_pc_observer_with_bound_op_copies_and_pickles(tmp_path):
    """An observer that has run the public-API step (its bound C++ op cached) deep-copies
    (ModelEMA, utils/util.py:386) and pickles (torch.save of a whole model): the copy runs
    on its own running state, and both continue exactly like an uncopied observer."""
    import copy
    g0 = torch.Generator(device=DEV).manual_seed(5)
    w1, w2 = (torch.randn(32, 8, 3, 3, device=DEV, generator=g0) * s for s in (0.05, 0.3))
    q = V.PerChannelUniformQuantizer(8, False)
    obs = V.PerChannelMinMaxObserver(False)
    obs.observe_quantize(w1.clone().requires_grad_(True), q)
    assert obs.__dict__.get("_op") is not None
    ref = copy.deepcopy(obs)   # the copy to compare with
    cp = copy.deepcopy(obs)
    path = tmp_path / "obs.pt"
    torch.save(obs, path)
    ld = torch.load(path, weights_only=False)   # our own file (written just above)
    for o in (cp, ld):
        assert "_op" not in o.__dict__ and o.run_min.data_ptr() != obs.run_min.data_ptr()
    y0, _ = obs.observe_quantize(w2.clone().requires_grad_(True), q)
    for o in (cp, ld, ref):
        y, _ = o.observe_quantize(w2.clone().requires_grad_(True), q)
        assert torch.equal(_bits(y), _bits(y0))
        assert torch.equal(_bits(o.run_max), _bits(obs.run_max))
        assert torch.equal(_bits(o.scale), _bits(obs.scale))


def test_pc_observer_bound_op_follows_a_replaced_run_max():
    """The bound op is keyed on BOTH running tensors: replacing run_max alone (a state
    restore, a sync that reassigns it) rebuilds it, so the next step updates and reads
    the new tensor -- equal to a fresh observer started from the same state."""
    g0 = torch.Generator(device=DEV).manual_seed(7)
    w1, w2 = (torch.randn(16, 8, 3, 3, device=DEV, generator=g0) * s for s in (0.05, 0.3))
    q = V.PerChannelUniformQuantizer(8, False)
    obs = V.PerChannelMinMaxObserver(False)
    obs.observe_quantize(w1.clone().requires_grad_(True), q)
    assert obs.__dict__.get("_op") is not None
    new_max = torch.full_like(obs.run_max, 5.0)
    obs.run_max = new_max
    ref = V.PerChannelMinMaxObserver(False)
    ref.run_min, ref.run_max = obs.run_min.clone(), new_max.clone()
    y, _ = obs.observe_quantize(w2.clone().requires_grad_(True), q)
    y_ref, _ = ref.observe_quantize(w2.clone().requires_grad_(True), q)
    assert obs.run_max is new_max and torch.all(new_max == 5.0)
    assert torch.equal(_bits(y), _bits(y_ref)) and torch.equal(_bits(obs.scale), _bits(ref.scale))


@pytest.mark.parametrize("act", [None, "relu", "silu"])
@pytest.mark.parametrize("kind", ["float", "cuda", "cpu", "qp"])
def test_fixed_ext_equals_python(kind, act, monkeypatch):
    g0 = torch.Generator(device=DEV).manual_seed(2)
    c = torch.randn(3, 8, 33, 17, device=DEV, generator=g0)
    g = torch.randn(c.shape, device=DEV, generator=g0)
    q = V.UniformQuantizer(4, False)
    scale, zp = 0.071, 5
    qp = torch.tensor([scale, zp, 0.0, 0.0], dtype=torch.float64, device=DEV)

    def run():
        x = c.clone().requires_grad_(True)
        if kind == "qp":
            y = V.fakequant.fake_quant_fixed(x, None, None, q.qmin, q.qmax, qp=qp, act=act)
        else:
            s = {"float": scale, "cuda": torch.tensor(scale, dtype=torch.float64, device=DEV),
                 "cpu": torch.tensor(scale, dtype=torch.float64)}[kind]
            y = q.quantize(x, s, zp, False, act=act)
        y.backward(g)
        return y, x.grad

    a, b = both(run, monkeypatch)
    for u, v in zip(a, b):
        assert torch.equal(_bits(u), _bits(v))


@pytest.mark.parametrize("act", [None, "relu"])
@pytest.mark.parametrize("where", ["cuda", "cpu"])
@pytest.mark.parametrize("asym", [False, True])
def test_learnable_ext_equals_python(asym, where, act, monkeypatch):
    g0 = torch.Generator(device=DEV).manual_seed(3)
    c = torch.randn(4, 16, 40, 40, device=DEV, generator=g0)
    g = torch.randn(c.shape, device=DEV, generator=g0)
    q = V.LSQQuantizer(8, False) if asym else V.UniformQuantizer(8, True)

    def run():
        x = c.clone().requires_grad_(True)
        s = torch.nn.Parameter(torch.tensor(0.03, dtype=torch.float64, device=where))
        z = torch.nn.Parameter(torch.tensor(3.4, dtype=torch.float64, device=where)) if asym else 0
        y = q.quantize(x, s, z, True, act=act)
        y.backward(g)
        out = [y, x.grad, s.grad]
        if asym:
            out.append(z.grad)
        return out

    a, b = both(run, monkeypatch)
    for u, v in zip(a, b):
        assert u.device == v.device and u.dtype == v.dtype and u.shape == v.shape
        assert torch.equal(_bits(u), _bits(v))


def test_lsq_fake_quantize_per_tensor_ext_equals_python(monkeypatch):
    g0 = torch.Generator(device=DEV).manual_seed(4)
    X = torch.randn(8, 16, 12, 12, device=DEV, generator=g0)
    g = torch.randn(X.shape, device=DEV, generator=g0)

    def run():
        torch.manual_seed(0)
        m = LSQFakeQuantize(learn_scale=True, config_act=True, observer=torch.ao.quantization.MinMaxObserver,
                            quant_min=0, quant_max=255).to(DEV)
        x = X.clone().requires_grad_(True)
        m(x.detach())            # observe -> scale / zp -> scale_param / zero_point_param_float
        m.disable_observer()
        y = m(x)
        y.backward(g)
        return [y, x.grad] + [p.grad for p in m.parameters() if p.grad is not None]

    a, b = both(run, monkeypatch)
    assert len(a) == len(b)
    for u, v in zip(a, b):
        assert torch.equal(_bits(u), _bits(v))


def test_public_api_host_cost_is_low():
    """The C2 step through the public API on the C++ nodes: one fwd+bwd per weight;
    reported for information (bench.py's api_us_per_step is the measured figure)."""
    import time
    w = (torch.randn(1024, 1024, 3, 3, device=DEV) * 0.05).requires_grad_(True)
    g = torch.randn_like(w)
    obs, q = V.PerChannelMinMaxObserver(False), V.PerChannelUniformQuantizer(8, False)
    for _ in range(10):
        w.grad = None
        y, _ = obs.observe_quantize(w, q)
        y.backward(g)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(100):
        w.grad = None
        y, _ = obs.observe_quantize(w, q)
        y.backward(g)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t) / 100 * 1e6
    print(f"public API C2 fwd+bwd: {us:.1f} us/step")
    assert np.isfinite(us)


@pytest.mark.parametrize("with_zp", [False, True])
def test_lsq_multi_ext_equals_python(with_zp, monkeypatch):
    """K7 (every learnable weight quantizer in one launch each way) as the C++ node
    LsqMultiBackward and as the Python FakeQuantLearnMultiFn: outputs, input gradients and
    every scale / zero-point gradient bit for bit; a host-number scale and an unused
    output (zero gradient) included."""
    from vsiquantization_amd.fakequant import LsqSpec, lsq_fake_quant_multi
    g0 = torch.Generator(device=DEV).manual_seed(3)
    shapes = [(16, 3, 3, 3), (32, 16, 3, 3), (600000,), (5, 7), (300000,)]   # 600000 > 2^19: K4 inside
    ws = [torch.randn(s, device=DEV, generator=g0) * 0.1 for s in shapes]
    gs = [torch.randn(s, device=DEV, generator=g0) for s in shapes]

    def run():
        xs = [w.clone().requires_grad_(True) for w in ws]
        scales = [torch.nn.Parameter(torch.tensor(0.02 + 0.01 * i, dtype=torch.float64, device=DEV))
                  for i in range(len(xs) - 1)] + [0.05]   # the last: a host number
        zp = torch.nn.Parameter(torch.tensor(2.0, dtype=torch.float64, device=DEV)) if with_zp else 0
        specs = [LsqSpec(s, zp if (with_zp and i == 1) else 0, 0 if (with_zp and i == 1) else -2,
                         15 if (with_zp and i == 1) else 1, (15 * x.numel()) ** -0.5, with_zp and i == 1)
                 for i, (x, s) in enumerate(zip(xs, scales))]
        ys = lsq_fake_quant_multi(xs, specs)
        loss = sum((y * g).sum() for y, g in zip(ys[:-1], gs[:-1]))   # the last output unused
        loss.backward()
        out = list(ys) + [x.grad for x in xs] + [s.grad for s in scales[:-1]]
        if with_zp:
            out.append(zp.grad)
        return out

    a, b = both(run, monkeypatch)
    assert len(a) == len(b)
    for u, v in zip(a, b):
        assert u is not None and v is not None
        assert torch.equal(_bits(u), _bits(v))
