"""Deterministic probe of the round-5 SIGABRT in a HIP-graph capture under RCCL
(profiles/r05/r05cap_rccl_capture.txt): which listed collective does ProcessGroupNCCL's
watchdog fail to poll while a capture is open?

Each mode runs in its own 1-rank process group (child process), issues an eager
collective and, without waiting for the watchdog (it reaps completed work only on its
~100 ms poll), opens a thread_local capture and holds it for 0.6 s, so several polls
land inside the capture:
  same      27 eager all_gathers on WORLD, 27 captured all_gathers on WORLD
  same_global  the same in global capture mode
  twin      eager all_reduce on WORLD, captured all_reduce on a second group that never
            ran a collective outside a capture
  nocoll    eager all_reduce on WORLD, capture holds only a torch kernel (no collective)
  twin_used the second group runs one eager collective first, then is captured
  recycle[_twin][:nocache]  see recycle(): eager works whose events were recorded under an
            earlier capture (torch's event cache), polled during a later capture
Prints one line per mode: rc and the watchdog's exception text."""
import os
import subprocess
import sys
import time


def child(mode):
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    twin = dist.new_group([0], backend="nccl", device_id=dev) if "twin" in mode else None
    if mode.startswith("recycle"):
        return recycle(mode, dev, twin)
    x = torch.ones(1024, device=dev)
    outs = [torch.empty(1024, device=dev) for _ in range(27)]
    if mode == "twin_used":
        for o in outs:
            dist.all_gather_into_tensor(o, x, group=twin)
    for o in outs:                         # 27 works listed on WORLD's watchdog (the act leg's step)
        dist.all_gather_into_tensor(o, x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cm = "global" if mode == "same_global" else "thread_local"
    with torch.cuda.graph(g, capture_error_mode=cm):
        for o in outs:
            x.mul_(1.0)
            if mode in ("same", "same_global"):
                dist.all_gather_into_tensor(o, x)
            elif mode in ("twin", "twin_used"):
                dist.all_gather_into_tensor(o, x, group=twin)
        time.sleep(0.6)                    # several watchdog polls inside the capture
    g.replay()
    torch.cuda.synchronize()
    time.sleep(0.3)
    print(f"CHILD_OK {mode} x0={float(x[0])}", flush=True)
    dist.destroy_process_group()


def recycle(mode, dev, twin):
    """capture #1 (27 all_gathers; their Work events come from torch's per-device event
    cache and go back to it), eager 27 all_gathers on WORLD (events taken from the cache
    -- possibly recorded under capture #1), then capture #2 on the same capture stream
    while the eager works are still listed."""
    import torch
    import torch.distributed as dist
    grp = twin if "twin" in mode else None
    x = torch.ones(1024, device=dev)
    outs = [torch.empty(1024, device=dev) for _ in range(27)]
    for o in outs:
        dist.all_gather_into_tensor(o, x, group=grp)   # warm-up: comm + stream ready
    torch.cuda.synchronize()
    time.sleep(0.5)
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, capture_error_mode="thread_local"):
        for o in outs:
            x.mul_(1.0)
            dist.all_gather_into_tensor(o, x, group=grp)
    torch.cuda.synchronize()
    for o in outs:                         # eager, WORLD: listed on WORLD's watchdog
        dist.all_gather_into_tensor(o, x)
    torch.cuda.synchronize()
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, capture_error_mode="thread_local"):
        for o in outs:
            x.mul_(1.0)
            dist.all_gather_into_tensor(o, x, group=grp)
        time.sleep(0.6)
    g1.replay()
    g2.replay()
    torch.cuda.synchronize()
    time.sleep(0.3)
    print(f"CHILD_OK {mode}", flush=True)
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        return child(sys.argv[2])
    modes = sys.argv[1:] or ["nocoll", "twin", "same", "twin_used", "same_global", "recycle", "recycle_twin",
                             "recycle:nocache", "recycle_twin:nocache"]
    for i, mm in enumerate(modes):
        m, _, opt = mm.partition(":")
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29611 + i), RANK="0",
                   WORLD_SIZE="1", LOCAL_RANK="0")
        if opt == "nocache":
            env["TORCH_NCCL_CUDA_EVENT_CACHE"] = "0"
        r = subprocess.run([sys.executable, "-u", __file__, "--child", m], env=env, capture_output=True,
                           text=True, timeout=120)
        why = [l.strip() for l in r.stderr.splitlines()
               if "exception" in l.lower() or "error" in l.lower() or "capture" in l.lower()][:12]
        ok = any(l.startswith("CHILD_OK") for l in r.stdout.splitlines())
        print(f"mode={mm} rc={r.returncode} ok={ok}", flush=True)
        for l in why:
            print(f"   {l[:400]}", flush=True)


if __name__ == "__main__":
    main()
