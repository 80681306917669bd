"""The host path's AVX-512 loops (csrc/host_simd.cpp) against its scalar loops
(VSIQ_HOST_SIMD=0, run in a child process): y, integer codes, masks, STE and LSQ grad_x,
the observer's min / max / NaN count and f64 sums, and the scale / zero-point gradient
sums, all bit for bit (the scalar loops accumulate in the AVX-512 loops' 16-lane order).
Lengths around the vector width and the 64K chunk; NaN, +-inf, -0.0, denormals and .5
ties in the data; no activation and fused ReLU."""
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.host_simd_cases import cases, run_case

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def scalar(tmp_path_factory):
    out = tmp_path_factory.mktemp("simd") / "scalar.npz"
    env = dict(os.environ, VSIQ_HOST_SIMD="0", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "host_simd_worker.py"), str(out)], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return np.load(out)


@pytest.mark.parametrize("name", list(cases()))
def test_simd_equals_scalar(scalar, name):
    from vsiquantization_amd import host
    if not host.simd():
        pytest.skip("this CPU has no AVX-512 F/BW/VL: the host path runs its scalar loops only")
    got = run_case(*cases()[name])
    for k, v in got.items():
        want = scalar[f"{name}.{k}"]
        if v.dtype.kind == "f":   # NaN payloads may differ (inf - inf vs a propagated NaN)
            nv, nw = np.isnan(v), np.isnan(want)
            assert np.array_equal(nv, nw), (name, k)
            v, want = np.where(nv, 0, v).astype(v.dtype), np.where(nw, 0, want).astype(want.dtype)
        assert np.array_equal(v.view(np.uint8), want.view(np.uint8)), (name, k, v, want)
