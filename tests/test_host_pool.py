"""The host path's thread pool (csrc/k_host.hip `Pool`) under back-to-back jobs: many
host calls of 4+ chunks each with VSIQ_HOST_THREADS far above the CPU count (workers
preempted between jobs -- the case where a worker still inside an earlier job could take
a chunk of the next one), from a child process so the variable is read at first use.
Every call must equal the single-threaded result bit for bit and none may hang."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from vsiquantization_amd import _hip as H
lib = H.lib()
assert lib.vsiq_host_threads() == 64, lib.vsiq_host_threads()
rng = np.random.default_rng(0)
n = 6 * 65536 + 11
x = torch.from_numpy((rng.standard_normal(n) * 2).astype(np.float32))
g = torch.from_numpy(rng.standard_normal(n).astype(np.float32))

def observe():
    st = torch.empty(H.ST_LEN, dtype=torch.float64); run = torch.zeros(2)
    qp = torch.empty(H.QP_LEN, dtype=torch.float64)
    assert lib.vsiq_host_observe_f32(H.ptr(x), H.c_i64(n), 0, H.ptr(st), H.ptr(run), H.ptr(qp), 0,
                                     255.00000001, 1e-8) == 0
    return st.numpy().copy()

def lsq():
    gx = torch.empty(n); go = torch.empty(2, dtype=torch.float64)
    assert lib.vsiq_host_lsq_bwd_f32(H.ptr(g), H.ptr(x), H.ptr(gx), H.c_i64(n), 1, 0.05, 3.0, 1, 0, 255,
                                     (255 * n) ** -0.5, H.ptr(go)) == 0
    return gx.numpy().copy(), go.numpy().copy()

def fq():
    y = torch.empty(n)
    assert lib.vsiq_host_fq_fwd_f32(H.ptr(x), H.ptr(y), None, None, H.c_i64(n), 0, None, 0.05, 0.0, 0, 0,
                                    -128, 127) == 0
    return y.numpy().copy()

def pc_observe(rows):
    # per-channel rows: the pool over rows (>= 4 rows) or, for fewer, inside each row
    # (nested Pool::run from inside a job must run serially, without the pool's mutex)
    w = x[: rows * (n // rows)].reshape(rows, -1).contiguous()
    run = torch.zeros(2, rows)
    s = torch.empty(rows, dtype=torch.float64); z = torch.empty(rows, dtype=torch.float64)
    y = torch.empty_like(w); st = torch.empty(rows, 3, dtype=torch.float64)
    assert lib.vsiq_host_pc_observe_fq_f32(H.ptr(w), H.ptr(y), None, H.c_i64(rows), H.c_i64(w.shape[1]),
                                           H.ptr(run[0]), H.ptr(run[1]), H.ptr(s), H.ptr(z), H.ptr(st), 0,
                                           255.00000001, 1e-8, 0, 255) == 0
    return [a.numpy().copy() for a in (y, s, z, st, run)]

s0, (gx0, go0), y0 = observe(), lsq(), fq()
pc0 = {r: pc_observe(r) for r in (2, 8)}
for it in range(400):
    assert np.array_equal(observe().view(np.uint8), s0.view(np.uint8)), it
    gx, go = lsq()
    assert np.array_equal(gx.view(np.uint8), gx0.view(np.uint8)) and np.array_equal(go, go0), it
    assert np.array_equal(fq().view(np.uint8), y0.view(np.uint8)), it
    if it % 20 == 0:
        for r, want in pc0.items():
            assert all(np.array_equal(a.view(np.uint8), b.view(np.uint8)) for a, b in zip(pc_observe(r), want)), (it, r)
print("POOL_OK")
'''


def test_pool_nested_rows_equal_single_thread():
    """Per-channel host rows with 2 rows (serial rows, the pool inside each) and 8 rows (the
    pool over rows, each row's own chunk loop serial inside it): bit-exact to one thread."""
    script = r'''
import sys, json, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from vsiquantization_amd import _hip as H
lib = H.lib()
rng = np.random.default_rng(1)
out = {}
for rows in (2, 8):
    w = torch.from_numpy((rng.standard_normal((rows, 5 * 65536 + 3)) * 2).astype(np.float32))
    run = torch.zeros(2, rows); s = torch.empty(rows, dtype=torch.float64); z = torch.empty(rows, dtype=torch.float64)
    y = torch.empty_like(w); st = torch.empty(rows, 3, dtype=torch.float64)
    assert lib.vsiq_host_pc_observe_fq_f32(H.ptr(w), H.ptr(y), None, H.c_i64(rows), H.c_i64(w.shape[1]),
                                           H.ptr(run[0]), H.ptr(run[1]), H.ptr(s), H.ptr(z), H.ptr(st), 0,
                                           255.00000001, 1e-8, 0, 255) == 0
    out[rows] = [float(y.double().sum()), s.tolist(), z.tolist(), st.reshape(-1).tolist(), run.reshape(-1).tolist(),
                 int(y.view(torch.int32).long().sum())]
print("OUT" + json.dumps(out))
'''
    res = {}
    for threads in ("1", "16"):
        env = dict(os.environ, VSIQ_HOST_THREADS=threads, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
        r = subprocess.run([sys.executable, "-c", script, ROOT], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
        res[threads] = next(l for l in r.stdout.splitlines() if l.startswith("OUT"))
    assert res["1"] == res["16"]


def test_pool_back_to_back_jobs_oversubscribed():
    env = dict(os.environ, VSIQ_HOST_THREADS="64", PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "POOL_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
