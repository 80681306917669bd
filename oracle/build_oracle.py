"""Build the oracle's C restatements (TEST INFRASTRUCTURE) into oracle/_build/.

`python -m oracle.build_oracle` or `__graft_entry__.build()`.  gcc only, no reference
sources involved: oracle/silu_ref.c restates torch's CPU SiLU arithmetic (Sleef /
glibc expf), oracle/mean_ref.c torch's CPU fp32 sum order (torch.mean), see their headers.  The .so is git-ignored and travels to the GPU box with
the tree like the product's own libraries.
"""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
OUTDIR = os.path.join(HERE, "_build")
SILU_SRC = os.path.join(HERE, "silu_ref.c")
SILU_LIB = os.path.join(OUTDIR, "libvsiq_oracle_silu.so")
MEAN_SRC = os.path.join(HERE, "mean_ref.c")
MEAN_LIB = os.path.join(OUTDIR, "libvsiq_oracle_mean.so")
FLAGS = ["-O2", "-ffp-contract=off", "-fno-builtin", "-fPIC", "-shared"]


def _build_one(src, out, force, verbose):
    if (not force and os.path.exists(out)
            and os.path.getmtime(out) >= os.path.getmtime(src)
            and os.path.getmtime(out) >= os.path.getmtime(__file__)):
        return out
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        raise RuntimeError("gcc not found: cannot build the oracle's C restatement")
    os.makedirs(OUTDIR, exist_ok=True)
    cmd = [cc, *FLAGS, "-o", out + ".tmp", src, "-lm"]
    if verbose:
        print("[oracle build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build(force: bool = False, verbose: bool = True) -> str:
    """Both restatements; returns the SiLU library's path (the mean one: build_mean())."""
    build_mean(force, verbose)
    return _build_one(SILU_SRC, SILU_LIB, force, verbose)


def build_mean(force: bool = False, verbose: bool = True) -> str:
    return _build_one(MEAN_SRC, MEAN_LIB, force, verbose)


if __name__ == "__main__":
    build(force=True)
