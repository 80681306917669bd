"""numpy restatement of the reference fake-quant arithmetic (TEST INFRASTRUCTURE).

Every function restates one reference op with IEEE fp32 element arithmetic
(numpy float32 true division, round-half-even ``np.rint``, NaN-propagating
clamp) and Python/float64 qparam math, in the reference's operation order.
Parity is pinned against goldens generated from the reference
(tests/golden/gen_goldens.py); see tests/test_oracle_golden.py.

Reference: tranngocduvnvp/VSIQuantization (/root/reference), arithmetic done by
PyTorch 2.10.0 CPU kernels (the reference pins no torch version; README.md:38).
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32


# --------------------------------------------------------------------------- ranges
def qrange(num_bits: int, symmetric: bool):
    """quantizers/uniform.py:24-32 — integer range of the quantizer."""
    if symmetric:
        return -(2 ** (num_bits - 1)), 2 ** (num_bits - 1) - 1
    return 0, 2 ** num_bits - 1


def grad_scale(qmax: int, numel: int, calib_grad_scale=1) -> float:
    """quantizers/uniform.py:58-71 (+ :48) — LSQ gradient scale (qmax*numel)^-1/2 * calib."""
    return ((qmax * numel) ** -0.5) * calib_grad_scale


# --------------------------------------------------------------------------- observer
def observe_minmax(x: np.ndarray, min_val=0, max_val=0):
    """observers/minmax.py:32-47 — running min/max update.

    ``x.min().item()`` is NaN when x holds a NaN; ``nan < v`` is False in Python,
    so a NaN-containing call leaves both bounds unchanged.  Strict comparisons:
    ``-0.0 < 0`` is False, so signed zeros never replace the initial int 0.
    An empty tensor raises in torch (min of empty); we mirror with ValueError.
    """
    x = np.asarray(x, dtype=F32)
    if x.size == 0:
        raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0")
    if np.isnan(x).any():
        min_x = max_x = float("nan")
    else:
        min_x = float(x.min())
        max_x = float(x.max())
    if min_val is None or min_x < min_val:
        min_val = min_x
    if max_val is None or max_x > max_val:
        max_val = max_x
    return min_val, max_val


def minmax_qparams(min_val, max_val, symmetric: bool, num_bits: int = 8, eps: float = 1e-8):
    """observers/minmax.py:49-74 — host float64 qparams (Python round = half-even,
    raises ValueError/OverflowError on NaN/inf exactly like the reference)."""
    if symmetric:
        max_abs = max(abs(min_val), abs(max_val))
        scale = max_abs / (2 ** (num_bits - 1) - 1 + eps)
        zero_point = 0
    else:
        scale = (max_val - min_val) / (2 ** num_bits - 1 + eps)
        zero_point = round(-min_val / (scale + eps))
    return scale, zero_point


# --------------------------------------------------------------------------- forward
def _clamp_nan(v: np.ndarray, qmin, qmax) -> np.ndarray:
    """torch.clamp on CPU: NaN propagates, -0.0 is kept (uniform.py:95)."""
    lo = F32(qmin)
    hi = F32(qmax)
    return np.where(v < lo, lo, np.where(v > hi, hi, v)).astype(F32)


def fq_codes(x, scale, zero_point, qmin, qmax):
    """quantizers/uniform.py:81-96 — ``clamp(round(x/scale + zp), qmin, qmax)``.

    ``scale``/``zero_point`` are Python numbers (or 0-dim f64 values): torch casts
    them to fp32 before the fp32 true division / add (x/py_float == x/f32(s)).
    Returns (x_int, in_range_mask) where the mask is evaluated on the ROUNDED
    value, inclusive (ClampBackward1 semantics).
    """
    x = np.asarray(x, dtype=F32)
    s = F32(scale)
    z = F32(zero_point)
    with np.errstate(all="ignore"):
        u = (x / s).astype(F32)
        u = (u + z).astype(F32)
        r = np.rint(u).astype(F32)
    mask = (r >= F32(qmin)) & (r <= F32(qmax))
    return _clamp_nan(r, qmin, qmax), mask


def fq_forward(x, scale, zero_point, qmin, qmax):
    """quantizers/uniform.py:54-56 — y = (x_int - zp) * scale (fp32)."""
    q, mask = fq_codes(x, scale, zero_point, qmin, qmax)
    with np.errstate(all="ignore"):
        y = ((q - F32(zero_point)).astype(F32) * F32(scale)).astype(F32)
    return y, q, mask


def fq_backward_fixed(g, mask, scale):
    """Autograd of uniform.py:54-55,95 with a Python-float scale (non-learnable):
    MulBackward (g*s) -> ClampBackward1 (mask) -> STE -> DivBackward (/s).
    grad_x = where(mask, g*s, 0) / s, all fp32."""
    g = np.asarray(g, dtype=F32)
    s = F32(scale)
    with np.errstate(all="ignore"):
        gq = (g * s).astype(F32)
        gm = np.where(mask, gq, F32(0.0)).astype(F32)
        return (gm / s).astype(F32)


def lsq_forward_backward(x, g, scale, zero_point, qmin, qmax, gscale, learn_zp=False):
    """Learnable path, quantizers/uniform.py:47-56 + torch autograd of the chain.

    scale: float64 value of the 0-dim Parameter (cast to fp32 in the forward).
    zero_point: 0 (symmetric / int) or the f64 value of a tensor zp (asym; then
    zp_eff = clamp(round(zp)) per uniform.py:98-102).
    learn_zp 2: a symmetric quantizer handed a gradient-requiring tensor zero point --
    uniform.py:50 skips zero_point_rounding and ScaleGradient, so zp enters x/s + zp and
    (x_int - zp) * s as given and its gradient carries no gscale factor.
    Returns y, grad_x, grad_scale (f64 closed form: f64 sums of the fp32 terms
    the reference sums in fp32), grad_zp (or None).
    """
    x = np.asarray(x, dtype=F32)
    g = np.asarray(g, dtype=F32)
    if learn_zp == 2:
        zp_eff = float(zero_point)
        zp_mask = True
    elif learn_zp:
        zr = float(np.rint(np.float64(zero_point)))
        zp_eff = min(max(zr, qmin), qmax)
        zp_mask = qmin <= zr <= qmax
    else:
        zp_eff = zero_point
        zp_mask = True
    s = F32(scale)
    z = F32(zp_eff)
    y, q, mask = fq_forward(x, scale, zp_eff, qmin, qmax)
    with np.errstate(all="ignore"):
        gq = (g * s).astype(F32)                                   # MulBackward0 (self)
        gm = np.where(mask, gq, F32(0.0)).astype(F32)              # ClampBackward1
        gx = (gm / s).astype(F32)                                  # DivBackward0 (self)
        t1 = (g * (q - z).astype(F32)).astype(F32)                 # MulBackward0 (other)
        xs = ((x / s).astype(F32) / s).astype(F32)
        t2 = ((-gm).astype(F32) * xs).astype(F32)                  # DivBackward0 (other)
    s1 = float(np.sum(t1, dtype=np.float64))
    s2 = float(np.sum(t2, dtype=np.float64))
    grad_s = (s1 + s2) * gscale
    grad_zp = None
    if learn_zp:
        a = float(np.sum(gm, dtype=np.float64))                    # AddBackward0 (other)
        b = float(np.sum(-gq, dtype=np.float64))                   # SubBackward0 (other)
        grad_zp = (a + b) if learn_zp == 2 else (((a + b) * gscale) if zp_mask else 0.0)
    return y, gx, grad_s, grad_zp


# --------------------------------------------------------------------------- per-channel LSQ (K6)
def pc_lsq_forward_backward(x, g, scales, zps, qmin, qmax, gscale, axis=1, learn_zp=True):
    """LSQFakeQuantize's learnable per-channel path (quantizers/lsq_module.py:134-166,
    314-343): every channel slice along ``axis`` is lsq_forward_backward with its own
    fp32 scale / rounded zero point; gradients per channel (f64 sums of fp32 terms).
    Returns y, grad_x, grad_scale [C], grad_zp [C]."""
    x = np.asarray(x, dtype=F32)
    g = np.asarray(g, dtype=F32)
    C = x.shape[axis]
    y = np.empty_like(x)
    gx = np.empty_like(x)
    gs = np.zeros(C)
    gz = np.zeros(C)
    for c in range(C):
        idx = [slice(None)] * x.ndim
        idx[axis] = c
        idx = tuple(idx)
        yc, gxc, gsc, gzc = lsq_forward_backward(x[idx], g[idx], float(scales[c]), float(zps[c]),
                                                 qmin, qmax, gscale, learn_zp=learn_zp)
        y[idx], gx[idx], gs[c] = yc, gxc, gsc
        gz[c] = gzc if gzc is not None else 0.0
    return y, gx, gs, gz


def lsq_module_grad_scale(x_shape, qmax, per_channel, config_act):
    """LSQFakeQuantize.calculate_grad_scale (lsq_module.py:314-333) x 5000 for activations
    (line 152): (quant_max * numel[/shape[1] if per-channel]) ** -0.5."""
    n = int(np.prod(x_shape))
    if per_channel:
        n /= x_shape[1]
    gs = (qmax * n) ** -0.5
    return gs * 5000 if config_act else gs


# --------------------------------------------------------------------------- fused activation (K5)
# F.silu on the reference's CPU tensors is torch's CPU silu kernel, whose exp is SLEEF's
# vectorized expf on most elements and glibc's scalar expf on the remainder of every
# parallel chunk; oracle/silu_ref.c restates both exps and the chunking (pinned against
# torch itself by tests/test_silu_oracle.py).  silu_ref = (W, threads) of the reference
# host: W = 2 x floats per vector (32 AVX-512, 16 AVX2, 0 = all on the vector path).
SILU_REF_DEFAULT = (32, 1)
_SILU = []


def _silu_lib():
    if not _SILU:
        import ctypes

        from oracle import build_oracle
        lib = ctypes.CDLL(build_oracle.build(verbose=False))
        P, I64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        lib.oracle_silu_fwd.argtypes = [P, P, I64, I, I, P]
        lib.oracle_silu_bwd.argtypes = [P, P, P, I64, I, I, P]
        lib.oracle_silu_scalar_map.argtypes = [P, I64, I, I]
        lib.oracle_exp_both.argtypes = [P, P, P, I64]
        _SILU.append(lib)
    return _SILU[0]


# --------------------------------------------------------------------------- mean|x| / mean x
# quantization_manager.py:66-67 records torch.mean(torch.abs(x)).cpu().item() and
# torch.mean(x): fp32 sums in torch's CPU cascade order, which depends on the host's
# thread count (oracle/mean_ref.c, pinned against torch.mean by tests/test_mean_oracle.py).
MEAN_REF_VEC = 8   # Vectorized<float> of the sum kernel this torch build dispatches (AVX2 and AVX-512)
_MEAN = []


def _mean_lib():
    if not _MEAN:
        import ctypes

        from oracle import build_oracle
        lib = ctypes.CDLL(build_oracle.build_mean(verbose=False))
        P, I64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        for f in (lib.oracle_torch_sum_f32, lib.oracle_torch_mean_f32):
            f.argtypes = [P, I64, I, I, I]
            f.restype = ctypes.c_float
        _MEAN.append(lib)
    return _MEAN[0]


def torch_mean(x, absf, threads, vec=MEAN_REF_VEC):
    """torch.mean(torch.abs(x)) (absf) or torch.mean(x) of a float32 array as torch's CPU
    kernel computes it on a host with `threads` threads: an np.float32."""
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32).reshape(-1))
    return np.float32(_mean_lib().oracle_torch_mean_f32(_p(a), a.size, int(bool(absf)), int(vec), int(threads)))


def torch_sum(x, absf, threads, vec=MEAN_REF_VEC):
    """The fp32 sum torch_mean divides (torch.sum on that host)."""
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32).reshape(-1))
    return np.float32(_mean_lib().oracle_torch_sum_f32(_p(a), a.size, int(bool(absf)), int(vec), int(threads)))


def _p(a):
    import ctypes
    return ctypes.c_void_p(a.ctypes.data)


def silu_forward(c, silu_ref=SILU_REF_DEFAULT):
    """torch CPU F.silu(c) on a host with layout silu_ref (flat element order)."""
    c = np.ascontiguousarray(c, dtype=F32)
    y = np.empty_like(c)
    sc = np.empty(max(c.size, 1), np.uint8)
    _silu_lib().oracle_silu_fwd(_p(c), _p(y), c.size, int(silu_ref[0]), int(silu_ref[1]), _p(sc))
    return y


def silu_backward(g, c, silu_ref=SILU_REF_DEFAULT):
    """torch CPU silu_backward(g, c) on a host with layout silu_ref."""
    g = np.ascontiguousarray(g, dtype=F32)
    c = np.ascontiguousarray(c, dtype=F32)
    gx = np.empty_like(c)
    sc = np.empty(max(c.size, 1), np.uint8)
    _silu_lib().oracle_silu_bwd(_p(g), _p(c), _p(gx), c.size, int(silu_ref[0]), int(silu_ref[1]), _p(sc))
    return gx


def silu_scalar_map(n, silu_ref=SILU_REF_DEFAULT):
    """bool[n]: elements torch's CPU kernel computes on its scalar (glibc expf) path."""
    sc = np.empty(max(n, 1), np.uint8)
    _silu_lib().oracle_silu_scalar_map(_p(sc), int(n), int(silu_ref[0]), int(silu_ref[1]))
    return sc[:n].astype(bool)


def exp_sleef_glibc(x):
    """(Sleef expf_u10(x), glibc expf(x)) of the restatement, for pinning."""
    x = np.ascontiguousarray(x, dtype=F32)
    a, b = np.empty_like(x), np.empty_like(x)
    _silu_lib().oracle_exp_both(_p(x), _p(a), _p(b), x.size)
    return a, b


def act_forward(c, act, silu_ref=SILU_REF_DEFAULT):
    """The fused layers' activation before quantize_out (modules/fused.py:133):
    F.relu (torch CPU: c < 0 -> +0, -0.0 and NaN pass through) or F.silu (torch CPU
    silu_kernel, bit for bit: silu_forward)."""
    c = np.asarray(c, dtype=F32)
    if act is None or act == "none":
        return c
    if act == "relu":
        return np.where(c < 0, F32(0.0), c).astype(F32)
    if act == "silu":
        return silu_forward(c, silu_ref).reshape(c.shape)
    raise ValueError(act)


def act_backward(g, c, act, silu_ref=SILU_REF_DEFAULT):
    """Autograd of act_forward: relu threshold_backward(g, relu(c), 0) = c <= 0 ? 0 : g
    (NaN passes g); silu_backward (g * sig) * fma(c, 1 - sig, 1) with the same exp split
    as the forward (silu_backward)."""
    g = np.asarray(g, dtype=F32)
    c = np.asarray(c, dtype=F32)
    if act is None or act == "none":
        return g
    if act == "relu":
        return np.where(c <= 0, F32(0.0), g).astype(F32)
    if act == "silu":
        return silu_backward(g, c, silu_ref).reshape(c.shape)
    raise ValueError(act)


# --------------------------------------------------------------------------- per-channel
def per_channel_observe_fq(w, symmetric: bool, bits: int, obs_bits: int = 8, eps: float = 1e-8,
                           run_min=None, run_max=None):
    """Per-channel (axis 0) observe + fake-quant, build-defined:
    ``for c: s_c, z_c = MinMaxObserver(sym, obs_bits).forward(W[c]);
    Y[c] = UniformQuantizer(bits, sym).quantize(W[c], s_c, z_c, False)``
    (observers/minmax.py:76-88, quantizers/uniform.py:34-56).

    run_min/run_max: optional per-channel running state (default fresh observers, 0/0).
    Returns dict with y, x_int, mask, scale (f64[C]), zp (int64[C]), min_val, max_val.
    """
    w = np.asarray(w, dtype=F32)
    C = w.shape[0]
    rows = w.reshape(C, -1)
    qmin, qmax = qrange(bits, symmetric)
    ys, qs, ms = np.empty_like(rows), np.empty_like(rows), np.empty(rows.shape, bool)
    scales = np.empty(C, np.float64)
    zps = np.empty(C, np.int64)
    mins = np.empty(C, np.float64)
    maxs = np.empty(C, np.float64)
    for c in range(C):
        mn = 0 if run_min is None else float(run_min[c])
        mx = 0 if run_max is None else float(run_max[c])
        mn, mx = observe_minmax(rows[c], mn, mx)
        s, z = minmax_qparams(mn, mx, symmetric, obs_bits, eps)
        y, q, m = fq_forward(rows[c], s, z, qmin, qmax)
        ys[c], qs[c], ms[c] = y, q, m
        scales[c], zps[c], mins[c], maxs[c] = s, z, mn, mx
    sh = w.shape
    return dict(y=ys.reshape(sh), x_int=qs.reshape(sh), mask=ms.reshape(sh), scale=scales,
                zp=zps, min_val=mins, max_val=maxs)


def per_channel_backward_fixed(g, mask, scales):
    """Per-channel STE backward: row c uses fp32(scale_c) (fq_backward_fixed per row)."""
    g = np.asarray(g, dtype=F32)
    C = g.shape[0]
    gr = g.reshape(C, -1)
    mr = np.asarray(mask).reshape(C, -1)
    out = np.empty_like(gr)
    for c in range(C):
        out[c] = fq_backward_fixed(gr[c], mr[c], scales[c])
    return out.reshape(g.shape)


# --------------------------------------------------------------------------- manager stats
def collect_stats(x):
    """quantizers/quantization_manager.py:66-68 — mean(|x|), mean(x), std(x) (unbiased).
    Computed in float64 here; the reference reduces in fp32 (tolerance, not bitwise)."""
    x = np.asarray(x, dtype=np.float64).ravel()
    n = x.size
    mean_abs = float(np.abs(x).sum() / n)
    mean = float(x.sum() / n)
    std = float(np.sqrt(((x - mean) ** 2).sum() / (n - 1))) if n > 1 else float("nan")
    return mean_abs, mean, std


def init_scale_for_learning(mean_abs_list, bits_width):
    """quantizers/quantization_manager.py:105-112."""
    return 2 * np.mean(mean_abs_list) / np.sqrt(2 ** (bits_width - 1) - 1)


def is_finite_number(v) -> bool:
    return isinstance(v, (int, float)) and math.isfinite(v)
