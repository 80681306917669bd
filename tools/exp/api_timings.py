"""bench.api_timings (public-API C2 step interleaved with torch's trivial step, learnable
per-call step vs torch's x * s), three times in one process.  usage: python tools/exp/api_timings.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_stream(torch.cuda.Stream(dev))
for r in range(3):
    t = bench.api_timings(dev)
    t["ratio_api_vs_torch"] = t["api_us_per_step"] / t["api_torch_ref_us_per_step"]
    print(json.dumps({k: round(v, 2) for k, v in t.items()}), flush=True)
