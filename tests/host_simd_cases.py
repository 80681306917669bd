"""Inputs for tests/test_host_simd.py: lengths around the 16-lane vector width and the
64K chunk, values that exercise every branch of the element code (NaN, +-inf, -0.0,
denormals, exact .5 ties after the division, both clamp edges)."""
import numpy as np
import torch

from vsiquantization_amd import _hip as H


def _data(n, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * 3).astype(np.float32)
    special = np.array([np.nan, np.inf, -np.inf, -0.0, 0.0, 1e-40, -1e-40, 0.25, -0.25, 0.75, 1000.0, -1000.0],
                       dtype=np.float32)
    k = min(n, 64)
    x[rng.choice(n, k, replace=False)] = rng.choice(special, k)
    g = rng.standard_normal(n).astype(np.float32)
    return x, g


def cases():
    out = {}
    for n in (1, 15, 16, 17, 1000, 65536 + 33, 4 * 65536 + 5):
        for act in (0, 1):
            out[f"n{n}_a{act}"] = (n, act)
    return out


def run_case(n, act):
    lib = H.lib()
    x, g = _data(n, n * 3 + act)
    xt, gt = torch.from_numpy(x), torch.from_numpy(g)
    res = {}
    st = torch.empty(H.ST_LEN, dtype=torch.float64)
    run = torch.zeros(2)
    qp = torch.empty(H.QP_LEN, dtype=torch.float64)
    assert lib.vsiq_host_observe_f32(H.ptr(xt), H.c_i64(n), act, H.ptr(st), H.ptr(run), H.ptr(qp), 0,
                                     255.00000001, 1e-8) == 0
    res["stats"] = st.numpy().copy()
    for s, z, lo, hi, disc in ((0.5, 0.0, -128, 127, 0), (0.05, 3.0, 0, 255, 0), (0.5, 0.0, -8, 7, 1)):
        y = torch.empty(n)
        codes = torch.empty(n, dtype=torch.uint8)
        mask = torch.empty(n, dtype=torch.uint8)
        assert lib.vsiq_host_fq_fwd_f32(H.ptr(xt), H.ptr(y), H.ptr(codes), H.ptr(mask), H.c_i64(n), act, None, s, z, 0,
                                        disc, lo, hi) == 0
        tag = f"{s}_{z}_{lo}_{disc}"
        res[f"y{tag}"], res[f"c{tag}"], res[f"m{tag}"] = y.numpy().copy(), codes.numpy().copy(), mask.numpy().copy()
        gx = torch.empty(n)
        assert lib.vsiq_host_ste_bwd_f32(H.ptr(gt), H.ptr(mask), H.ptr(xt), H.ptr(gx), H.c_i64(n), act, s) == 0
        res[f"ste{tag}"] = gx.numpy().copy()
        go = torch.empty(2, dtype=torch.float64)
        assert lib.vsiq_host_lsq_bwd_f32(H.ptr(gt), H.ptr(xt), H.ptr(gx), H.c_i64(n), act, s, z, int(z != 0.0), lo, hi,
                                         (hi * n) ** -0.5, H.ptr(go)) == 0
        res[f"lsq{tag}"], res[f"lsqg{tag}"] = gx.numpy().copy(), go.numpy().copy()
    return res
