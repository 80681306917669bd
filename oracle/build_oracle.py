"""Build the oracle's C restatements (TEST INFRASTRUCTURE) into oracle/_build/.

`python -m oracle.build_oracle` or `__graft_entry__.build()`.  gcc only, no reference
sources involved: oracle/silu_ref.c restates torch's CPU SiLU arithmetic (Sleef /
glibc expf), see its header.  The .so is git-ignored and travels to the GPU box with
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
FLAGS = ["-O2", "-ffp-contract=off", "-fno-builtin", "-fPIC", "-shared"]


def build(force: bool = False, verbose: bool = True) -> str:
    if (not force and os.path.exists(SILU_LIB)
            and os.path.getmtime(SILU_LIB) >= os.path.getmtime(SILU_SRC)
            and os.path.getmtime(SILU_LIB) >= os.path.getmtime(__file__)):
        return SILU_LIB
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        raise RuntimeError("gcc not found: cannot build the oracle's C restatement")
    os.makedirs(OUTDIR, exist_ok=True)
    cmd = [cc, *FLAGS, "-o", SILU_LIB + ".tmp", SILU_SRC, "-lm"]
    if verbose:
        print("[oracle build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(SILU_LIB + ".tmp", SILU_LIB)
    return SILU_LIB


if __name__ == "__main__":
    build(force=True)
