"""One line per config of a bench.py JSON line: value, ms/step, kernel fracs (graph and
direct launch), API timings.  Usage: python tools/summarize_bench.py <file with the JSON line>"""
import json
import sys


def line(name, d):
    k = ", ".join(f"{n} {v['avg_us']:.1f}us {v['frac']:.3f}" for n, v in d.get("kernels", {}).items()
                  if isinstance(v, dict) and "frac" in v)
    dr = d.get("alt_launch")
    extra = (f" | {d.get('launch', '?')[:5]}; alt {dr['launch'][:5]} {dr['value']:.0f} {1e3 * dr['ms_per_step']:.1f}us"
             f" frac {dr['frac']:.3f}") if dr else ""
    cb = d.get("cpu_baseline", {}).get("value")
    return f"{name:5s} {d['value']:12.1f} Melem/s {1e3 * d['ms_per_step']:9.2f} us/step  [{k}]{extra}" + (
        f" cpu {cb:.1f}" if cb else "")


for path in sys.argv[1:]:
    txt = [l for l in open(path) if l.lstrip().startswith("{")]
    d = json.loads(txt[-1])
    print(line(d["config"].get("workload", "?")[:5], d))
    for k, v in (d.get("configs") or {}).items():
        print(line(k, v))
    if "batched_act_quant" in d:
        print(line("act", d["batched_act_quant"]))
    for k in ("api_us_per_step", "api_us_per_step_min", "api_graph_us_per_step"):
        if k in d:
            print(f"{k} {d[k]}")
    print("roofline", d["roofline"])
