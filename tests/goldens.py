"""Loader + comparison helpers for the reference golden vectors (tests/golden/)."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN_DIR = os.path.join(HERE, "golden")

_cache = {}


def load():
    if "d" not in _cache:
        with open(os.path.join(GOLDEN_DIR, "cases.json")) as f:
            meta = json.load(f)
        arrs = np.load(os.path.join(GOLDEN_DIR, "fakequant_goldens.npz"), allow_pickle=False)
        _cache["d"] = (meta["cases"], {k: arrs[k] for k in arrs.files})
    return _cache["d"]


def cases(kind):
    cs, _ = load()
    return [c for c in cs if c.get("kind") == kind]


def arr(key):
    _, a = load()
    return a[key]


def assert_bitwise_f32(got, want, what=""):
    """Bit-exact fp32 equality; NaNs must coincide (payload/sign of NaN ignored:
    x86 produces the negative default NaN, CDNA the positive one)."""
    got = np.asarray(got, dtype=np.float32)
    want = np.asarray(want, dtype=np.float32)
    assert got.shape == want.shape, f"{what}: shape {got.shape} vs {want.shape}"
    gn, wn = np.isnan(got), np.isnan(want)
    assert np.array_equal(gn, wn), f"{what}: NaN positions differ ({int((gn ^ wn).sum())} elems)"
    gb = got.view(np.uint32)[~gn]
    wb = want.view(np.uint32)[~wn]
    bad = np.flatnonzero(gb != wb)
    if bad.size:
        i = bad[0]
        raise AssertionError(f"{what}: {bad.size} of {gb.size} elements differ bitwise; first: "
                             f"got {got[~gn][i]!r} want {want[~wn][i]!r}")


def unpack_mask(words, rows, rowlen):
    """1-bit straight-through mask (include/vsiq.h layout) -> bool [rows, rowlen]."""
    W = 4 * -(-rowlen // 256)
    w = np.asarray(words).view(np.uint64)[: rows * W].reshape(rows, W)
    e = np.arange(rowlen)
    word = 4 * (e // 256) + (e % 4)
    bit = ((e % 256) // 4).astype(np.uint64)
    return ((w[:, word] >> bit) & np.uint64(1)).astype(bool)


def assert_close_f32(got, want, what="", rtol=1e-5, atol=1e-6):
    """Toleranced fp32 comparison for SiLU paths (exp differs by ~1 ulp between
    torch's CPU Sleef exp, numpy and the GPU); NaNs must coincide."""
    got = np.asarray(got, dtype=np.float32)
    want = np.asarray(want, dtype=np.float32)
    assert got.shape == want.shape, f"{what}: shape {got.shape} vs {want.shape}"
    gn, wn = np.isnan(got), np.isnan(want)
    assert np.array_equal(gn, wn), f"{what}: NaN positions differ ({int((gn ^ wn).sum())} elems)"
    ok = np.isclose(got[~gn], want[~wn], rtol=rtol, atol=atol)
    assert ok.all(), (f"{what}: {int((~ok).sum())} of {ok.size} elements beyond rtol={rtol} "
                      f"atol={atol}; max abs diff {np.max(np.abs(got[~gn] - want[~wn]))}")


def assert_fq_close(got, want, scale, what="", max_frac=0.01):
    """SiLU + fake quant: the codes may move by one step where silu(c) itself sits on
    a rounding boundary (a 1-ulp exp difference); everything else bitwise."""
    got = np.asarray(got, dtype=np.float32)
    want = np.asarray(want, dtype=np.float32)
    gn, wn = np.isnan(got), np.isnan(want)
    assert np.array_equal(gn, wn), f"{what}: NaN positions differ"
    d = np.abs(got[~gn].astype(np.float64) - want[~wn].astype(np.float64))
    bad = d > 0
    assert (d <= float(np.float32(scale)) * 1.0001 + 1e-12).all(), f"{what}: a code moved by > 1 step"
    assert bad.mean() <= max_frac, f"{what}: {bad.mean():.4f} of elements moved a step"
