"""bench.py host logic (no GPU): workload shapes match SURVEY.md §8 configs, the N-rank
launcher, the CPU-baseline thread plan."""
import json
import os
import subprocess
import sys

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_yolov8n_backbone_matches_survey_c4():
    layers = bench.yolov8n_backbone()
    assert len(layers) == 27
    assert sum(co * h * h for _, co, _, _, h in layers) == 2_137_600      # act elem / image
    assert sum(ci * co * k * k for ci, co, k, _, _ in layers) == 1_267_632   # weight elems
    assert layers[0] == (3, 16, 3, 2, 160) and layers[-1] == (512, 256, 1, 1, 10)


def test_parse_extras_defaults():
    assert bench.parse([]).extras == ["c1", "c3", "c4", "c5", "act"]          # headline C2: all configs
    assert bench.parse(["--workload", "c3"]).extras == []
    assert bench.parse(["--extras", "none"]).extras == []
    assert bench.parse(["--extras", "c4,act"]).extras == ["c4", "act"]


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=240)


def test_gpus_2_spawns_two_ranks():
    """--gpus 2 without torchrun: the launcher starts torch.distributed.run with 2 ranks
    (gloo rehearsal of the rendezvous, no GPU) and rank 0 reports the world size."""
    p = _run(["--gpus", "2", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert out == {"dry_run": True, "n_gpus": 2, "requested_gpus": 2, "ranks_joined": 2}


def test_world_size_mismatch_is_an_error():
    p = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr


def test_cpu_thread_counts_start_with_os_cpu_count():
    counts, total, usable = bench.cpu_thread_counts()
    assert counts[0] == total == os.cpu_count()
    assert 1 <= usable <= total and len(set(counts)) == len(counts)


def test_cpu_baseline_c1_reports_threads():
    r = bench.cpu_baseline("c1", 0.2)
    assert r["kind"] == "port" and r["value"] > 0 and r["unit"] == "Melem/s"
    assert str(os.cpu_count()) in r["thread_probe_c1"] and str(r["cores"]) in r["threads_whole"]


def _settle_worker(rank, world, port, ret):
    """settle_gates with a step that holds a collective and a tuner that reports nothing
    pending from its 2nd query on rank 0 but only from its 4th on rank 1: the agreed
    stop keeps the ranks in step."""
    import torch
    import torch.distributed as dist
    from vsiquantization_amd import _hip as H
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rounds = {"n": 0}

    def pending():
        rounds["n"] += 1
        return 0 if rounds["n"] > (1 if rank == 0 else 3) else 5

    class W:
        def launch(self, i):
            t = torch.ones(1)
            dist.all_reduce(t)              # the step's collective
            return 0 if float(t) == world else 1
    H.gate_tuning_pending = pending
    torch.cuda.synchronize = lambda *a: None
    try:
        ret[rank] = bench.settle_gates(W(), world=world)[0]
    finally:
        dist.destroy_process_group()


def test_settle_gates_agrees_across_ranks():
    import torch.multiprocessing as mp
    port = 29700 + os.getpid() % 200
    ret = mp.Manager().dict()
    mp.spawn(_settle_worker, args=(2, port, ret), nprocs=2, join=True)
    assert ret[0] == ret[1] == 32          # 4 rounds of 8 steps on both ranks


def _agree_worker(rank, world, port, ret):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ret[rank] = (bench._agree(True, world), bench._agree(rank == 0, world), bench._agree(False, world))
    finally:
        dist.destroy_process_group()


def test_launch_mode_agreed_across_ranks():
    """measure()'s capture / graph choice is agreed (all-reduce MIN): graphs only when
    every rank captured and every rank's trial chose them."""
    import torch.multiprocessing as mp
    port = 29900 + os.getpid() % 90
    ret = mp.Manager().dict()
    mp.spawn(_agree_worker, args=(2, port, ret), nprocs=2, join=True)
    assert ret[0] == ret[1] == (True, False, False)


def test_compact_summary_is_short_and_complete():
    """The stderr summary after the JSON line carries every leg's value, kernel fractions
    (off-step kernels marked *), API timings and chosen gates in a few hundred characters."""
    k = {"pc_observe_fq_fwd": {"frac": 0.74, "avg_us": 12.9}, "ste_bwd": {"frac": 0.76, "avg_us": 12.4},
         "alt": {"frac": 0.8, "avg_us": 1.0, "in_step": False}}
    leg = {"value": 1000.0, "ms_per_step": 0.2, "launch": "direct", "kernels": k}
    out = dict(leg, config={"workload": "C2 per-channel"}, configs={"c5": dict(leg)}, batched_act_quant=dict(leg),
               api_us_per_step=50.0, api_torch_ref_us_per_step=45.0,
               store_gate={"sites": [{"site": "k3", "gate_ticks": 515}]}, cpu_baseline={"value": 100.0})
    s = bench.compact_summary(out)
    assert s.startswith("[bench summary]") and len(s) < 1500
    assert "pc_observe_fq_fwd=0.740" in s and "alt=0.800*" in s and "k3:515" in s and "api_us_per_step" in s
    assert "c5 " in s and "act " in s and "cpu=100.0" in s
    out["store_gate"]["sites"][0]["candidates"] = [[0, 13.41], [489, 12.93], [515, 12.71], [541, 12.80]]
    assert "k3:515(12.71/13.41us)" in bench.compact_summary(out)
    out["configs"]["c4"] = {"metric": "m", "error": "RuntimeError('x')"}   # a failed secondary leg
    assert "c4 FAILED RuntimeError('x')" in bench.compact_summary(out)


def test_gate_report_candidates_parsed(monkeypatch):
    """settle_gates keeps every timed candidate of a site ([ticks, median us])."""
    from vsiquantization_amd import _hip as H
    rep = "k3_pc_observe_fq dev=0 grid=1024 bytes=37748736 est=503 done=1 best=528 retunes=1 watch=256 0:13.41 453:12.95 528:12.70\n"
    monkeypatch.setattr(H, "gate_tuning_pending", lambda: 0)
    monkeypatch.setattr(H, "gate_report", lambda: rep)
    monkeypatch.setattr(bench.torch.cuda, "synchronize", lambda *a: None)

    class W:
        def launch(self, i):
            return 0
    n, sites = bench.settle_gates(W())
    assert n == 8 and sites[0]["gate_ticks"] == 528 and sites[0]["retunes"] == 1
    assert sites[0]["candidates"] == [[0, 13.41], [453, 12.95], [528, 12.70]]


def test_chained_group_events_durations():
    """Consecutive launch groups share their boundary event (bench._Chained): per-phase
    durations read from the chained rows equal those of separate events per group."""
    class Ev:
        def __init__(self, t):
            self.t = t

        def record(self, *_):
            pass

        def elapsed_time(self, end):
            return end.t - self.t
    # 3 groups x 2 phases: boundaries at 0, 5, 9 | 9, 14, 20 | 20, 26, 30 (ms)
    marks = [[0, 5, 9], [9, 14, 20], [20, 26, 30]]
    rows = []
    for m in marks:
        row = [Ev(t) for t in m]
        if rows:
            row[0] = bench._Chained(rows[-1][-1])
        rows.append(row)
    assert rows[1][0].record() is None   # recording the shared event again is a no-op
    d = bench._durations(rows, ["fwd", "bwd"], steps=1000)
    assert d == {"fwd": (5 + 5 + 6) / 1000 * 1e-3, "bwd": (4 + 6 + 4) / 1000 * 1e-3}
