"""Loader + comparison helpers for the reference golden vectors (tests/golden/)."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN_DIR = os.path.join(HERE, "golden")

_cache = {}

# The reference host the goldens were generated on (tests/golden/gen_goldens.py, the build
# container): torch CPU kernels AVX-512 (W = 32 elements per vectorized SiLU step), 8
# threads.  Every golden tensor is below torch's 32768-element grain, so only W matters.
GOLDEN_SILU_REF = (32, 8)


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
    """Toleranced fp32 comparison (floats the reference does not pin bitwise, e.g. MIOpen's
    weight gradient); NaNs must coincide."""
    got = np.asarray(got, dtype=np.float32)
    want = np.asarray(want, dtype=np.float32)
    assert got.shape == want.shape, f"{what}: shape {got.shape} vs {want.shape}"
    gn, wn = np.isnan(got), np.isnan(want)
    assert np.array_equal(gn, wn), f"{what}: NaN positions differ ({int((gn ^ wn).sum())} elems)"
    ok = np.isclose(got[~gn], want[~wn], rtol=rtol, atol=atol)
    assert ok.all(), (f"{what}: {int((~ok).sum())} of {ok.size} elements beyond rtol={rtol} "
                      f"atol={atol}; max abs diff {np.max(np.abs(got[~gn] - want[~wn]))}")
