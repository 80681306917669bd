"""Build the in-tree HIP shared library (gfx950) — `python -m vsiquantization_amd._build`.

One translation unit, compiled by hipcc straight into `_vsiq_hip.so` next to this
file, so the built library travels with the repository snapshot to the GPU box.
Flags that matter for parity with the reference's CPU arithmetic:
  -ffp-contract=off                       no FMA contraction of (q - zp) * s etc.
  -fhip-fp32-correctly-rounded-divide-sqrt   IEEE x / s
  -fno-gpu-flush-denormals-to-zero        keep fp32 denormals (torch CPU keeps them)
  -mcode-object-version=5                 loadable by torch's bundled ROCm 7.0 runtime
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "vsiq_kernels.hip")
OUT = os.path.join(HERE, "_vsiq_hip.so")
ARCH = os.environ.get("VSIQ_OFFLOAD_ARCH", "gfx950")

FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    "-ffp-contract=off",
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-fno-gpu-flush-denormals-to-zero",
    "-mcode-object-version=5",
    "-Wall",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build vsiquantization_amd)")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [SRC, os.path.join(ROOT, "include", "vsiq.h"), __file__]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not needs_build():
        return OUT
    cmd = [hipcc(), *FLAGS, "-I", os.path.join(ROOT, "include"), "-o", OUT + ".tmp", SRC]
    if verbose:
        print("[vsiq build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
