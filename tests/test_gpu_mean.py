"""K11 (csrc/k_mean.hip): the reference's per-call mean|x| / mean x (quantization_manager.py
:66-67, torch.mean on the reference host's CPU) bit for bit on the GPU, against the
oracle (oracle/mean_ref.c, pinned to torch.mean by tests/test_mean_oracle.py):

* every layout boundary (vector, row, level step, GRAIN_SIZE, chunk) at 1 / 3 / 8 / 16
  reference threads, activations none / ReLU / SiLU (with its own reference layout);
* C5-sized layers (3.3M, 13.1M elements) and a 52M-element tensor, whose chunks pass the
  level-step change (B = 32 rows: one thread), NaN / inf;
* through QuantizationManager under H.set_mean_reference: per-call, deferred
  (calibrate_qat_model's K2o records) and observe+quantize calls record the oracle's means.
"""
import numpy as np
import pytest
import torch

from vsiquantization_amd import _hip as H
from vsiquantization_amd.fakequant import torch_mean
from oracle import fakequant_np as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SIZES = [0, 1, 7, 8, 9, 33, 513, 8191, 8193, 32767, 32768, 32769, 65537, 262_144, 1_000_003]


def _x(n, seed):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal(n) * rng.uniform(0.1, 10)).astype(np.float32)


def _same(a, b):
    a, b = np.float32(a), np.float32(b)
    return (np.isnan(a) and np.isnan(b)) or a.tobytes() == b.tobytes()


def _check(x, act, threads, silu_ref=(32, 8)):
    actv = H.SiluAct(*silu_ref) if act == "silu" else act
    got = torch_mean(torch.from_numpy(x).to(DEV), act=actv, ref=(8, threads)).cpu().numpy()
    a = O.act_forward(x, act, silu_ref) if act else x
    for j, absf in enumerate((1, 0)):
        assert _same(got[j], O.torch_sum(a, absf, threads)), (x.size, act, threads, absf, "sum")
        assert _same(got[2 + j], O.torch_mean(a, absf, threads)), (x.size, act, threads, absf, "mean")


@pytest.mark.parametrize("act", [None, "relu", "silu"])
@pytest.mark.parametrize("threads", [1, 3, 8, 16])
def test_k11_equals_oracle(act, threads):
    for i, n in enumerate(SIZES):
        _check(_x(n, 31 * threads + i), act, threads)


@pytest.mark.parametrize("n,threads", [(3_276_800, 8), (13_107_200, 8), (13_107_200, 16), (52_428_800, 1),
                                       (52_428_800, 8)])
def test_k11_large(n, threads):
    _check(_x(n, n % 9973), "relu" if threads == 8 else None, threads)


def test_k11_specials():
    x = _x(300_001, 5)
    x[[3, 40_000, 300_000]] = [np.inf, -0.0, 1e-40]
    _check(x, None, 8)
    x[77] = np.nan
    got = torch_mean(torch.from_numpy(x).to(DEV), ref=(8, 8)).cpu().numpy()
    assert np.isnan(got).all()


def test_k11_stats_record_and_errors():
    x = torch.from_numpy(_x(5000, 1)).to(DEV)
    st = torch.zeros(H.ST_LEN, dtype=torch.float64, device=DEV)
    nb = int(H.lib().vsiq_torch_mean_ws_bytes(5000, 8, 8))
    ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
    rc = H.lib().vsiq_torch_mean_f32(H.ptr(x), 5000, 0, 8, 8, None, H.ptr(st), H.ptr(ws), nb, H.stream_of(x.device))
    assert rc == 0
    xs = x.cpu().numpy()
    assert float(st[H.ST_MEANABS]) == float(O.torch_mean(xs, 1, 8))
    assert float(st[H.ST_MEAN]) == float(O.torch_mean(xs, 0, 8))
    torch.cuda.synchronize()
    assert float(st[H.ST_MIN]) == 0.0   # nothing else written
    assert H.lib().vsiq_torch_mean_ws_bytes(5000, 4, 8) == -1
    assert H.lib().vsiq_torch_mean_f32(H.ptr(x), 5000, 0, 8, 8, None, H.ptr(st), H.ptr(ws), nb - 1,
                                       H.stream_of(x.device)) != 0


@pytest.mark.parametrize("path", ["per_call", "deferred_relu", "observe_quantize"])
def test_manager_records_reference_means(path):
    """QuantizationManager under set_mean_reference(8): every recorded mean|x| / mean x is
    the oracle's for that call (the deferred K2o calls too, folded at the read)."""
    import vsiquantization_amd as V
    H.set_mean_reference(8)
    try:
        qm = V.QuantizationManager("UniformQuantizer", "MinMaxObserver", 4, True, is_learning_scale=False)
        qm.is_quantize = path == "observe_quantize"
        qm.dist_defer = path == "deferred_relu"
        xs = [_x(n, 70 + n % 13) for n in (600, 40_000, 1_200_000)]
        want_a, want_s = [], []
        for x in xs:
            t = torch.from_numpy(x).to(DEV)
            if path == "deferred_relu":
                qm.quantize(t, act="relu")
                a = O.act_forward(x, "relu")
            else:
                qm.quantize(t)
                a = x
            want_a.append(float(O.torch_mean(a, 1, 8)))
            want_s.append(float(O.torch_mean(a, 0, 8)))
        assert [float(v) for v in qm.mean_abs_x] == want_a
        assert [float(v) for v in qm.mean_x] == want_s
        want_sd = [float(_std_ref(O.act_forward(x, "relu") if path == "deferred_relu" else x, 8)) for x in xs]
        assert [float(v) for v in qm.std] == want_sd
    finally:
        H.clear_mean_reference()


def _std_ref(a, threads):
    """torch.std(a) on a reference host of `threads` threads (tests/test_mean_oracle.py
    pins this restatement against torch.std): the fp32 mean of that layout as a double,
    the f64 sum of squared deviations / (n - 1), sqrt, rounded to fp32."""
    if a.size < 2:
        return np.float32(np.nan)
    m = float(O.torch_mean(a, 0, threads))
    return np.float32(np.sqrt(np.sum((a.astype(np.float64) - m) ** 2) / (a.size - 1)))


@pytest.mark.parametrize("act", [None, "relu", "silu"])
def test_k11_std_pass(act):
    """vsiq_torch_mean_f32 with a stats record: VSIQ_ST_STD is torch.std(act(x)) of the
    reference host, bit for bit (fakequant.torch_stats)."""
    from vsiquantization_amd.fakequant import torch_stats
    for i, n in enumerate([1, 2, 9, 600, 32769, 1_000_003, 13_107_200]):
        x = _x(n, 900 + i)
        actv = H.SiluAct(32, 8) if act == "silu" else act
        got = torch_stats(torch.from_numpy(x).to(DEV), act=actv, ref=(8, 8)).cpu().numpy()
        a = O.act_forward(x, act, (32, 8)) if act else x
        assert _same(got[0], O.torch_mean(a, 1, 8)) and _same(got[1], O.torch_mean(a, 0, 8)), (n, act)
        assert _same(got[2], _std_ref(a, 8)), (n, act, got[2], _std_ref(a, 8))
    x = _x(5000, 3)
    x[17] = np.inf
    assert np.isnan(torch_stats(torch.from_numpy(x).to(DEV), ref=(8, 8)).cpu().numpy()[2])
