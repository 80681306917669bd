"""Host (CPU-tensor) path speed: the C ABI host loops at 64K..16M elements with 1 thread
and with the pool (VSIQ_HOST_THREADS is read once per process, so each setting runs in
a child), scalar vs AVX-512, and BASELINE C1 through the product vs the reference's
eager op sequence (oracle/eager_torch.py) at torch's thread count."""
import os
import subprocess
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")

CHILD = r'''
import time, torch, resource
from vsiquantization_amd import host, _hip as H
lib = H.lib()
out = []
for n in (65536, 1 << 20, 1 << 24):
    x = torch.randn(n, generator=torch.Generator().manual_seed(0))
    y = torch.empty_like(x); st = torch.empty(H.ST_LEN, dtype=torch.float64); run = torch.zeros(2)
    qp = torch.empty(H.QP_LEN, dtype=torch.float64)
    def t(fn, N=max(10, 4000000 // n)):
        for _ in range(3): fn()
        t0 = time.perf_counter()
        for _ in range(N): fn()
        return (time.perf_counter() - t0) / N * 1e6
    o = t(lambda: lib.vsiq_host_observe_f32(H.ptr(x), H.c_i64(n), 0, H.ptr(st), H.ptr(run), H.ptr(qp), 1, 127.00000001, 1e-8))
    f = t(lambda: lib.vsiq_host_fq_fwd_f32(H.ptr(x), H.ptr(y), None, None, H.c_i64(n), 0, None, 0.02, 0.0, 0, 0, -128, 127))
    out.append(f"n={n}: observe {o:.1f} us ({n / o:.0f} Melem/s), fq {f:.1f} us ({n / f:.0f} Melem/s)")
print(f"threads={host.threads()} " + "; ".join(out))
'''

C1 = r'''
import time, torch
import vsiquantization_amd as V
from oracle import eager_torch as E
from oracle.fakequant_np import minmax_qparams
x = torch.randn(256, 256, generator=torch.Generator().manual_seed(0))
q = V.UniformQuantizer(8, True)
def prod():
    s, z = V.MinMaxObserver(True).forward(x)
    return q.quantize(x, s, z, False)
def ref():
    mn, mx = E.observe(x); s, z = minmax_qparams(mn, mx, True, 8); return E.fake_quant(x, s, z, -128, 127)
def t(fn, N=400):
    for _ in range(20): fn()
    best = 1e9
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(N // 5): fn()
        best = min(best, (time.perf_counter() - t0) / (N // 5) * 1e6)
    return best
print(f"C1 256x256 per call: product host path {t(prod):.1f} us, reference eager {t(ref):.1f} us at {torch.get_num_threads()} torch threads")
'''


def main():
    env0 = dict(os.environ, PYTHONPATH=ROOT)
    for extra in ({"VSIQ_HOST_THREADS": "1", "VSIQ_HOST_SIMD": "0"}, {"VSIQ_HOST_THREADS": "1"}, {}):
        r = subprocess.run([sys.executable, "-c", CHILD], env=dict(env0, **extra), capture_output=True, text=True,
                           timeout=600)
        print(extra or "default", r.stdout.strip() or r.stderr[-2000:], flush=True)
    r = subprocess.run([sys.executable, "-c", C1], env=env0, cwd=ROOT, capture_output=True, text=True, timeout=600)
    print(r.stdout.strip() or r.stderr[-2000:], flush=True)


if __name__ == "__main__":
    main()
