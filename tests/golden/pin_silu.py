"""Exhaustive pin of the oracle's SiLU restatement (oracle/silu_ref.c) -- run by hand,
~10 minutes on 8 cores; the result is recorded in DESIGN.md §2.1.

1. oracle_glibc_expf vs this host's libm expf (the reference's scalar-path exp), all
   2^32 inputs, in a compiled C driver (ctypes per element would take days).
2. oracle silu (W = 2 x vector width, every element on the vectorized path) vs
   torch.nn.functional.silu on CPU over all 2^32 inputs, in chunks of 2^26 (a multiple
   of W per thread chunk, so torch runs every element through Sleef's expf).

Usage: python tests/golden/pin_silu.py
"""
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import fakequant_np as O  # noqa: E402

DRIVER = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
float oracle_glibc_expf(float);
int main(void) {
  uint64_t bad = 0;
  for (uint64_t u = 0; u < (1ULL << 32); ++u) {
    uint32_t b = (uint32_t)u; float x; memcpy(&x, &b, 4);
    float a = expf(x), c = oracle_glibc_expf(x);
    uint32_t ua, uc; memcpy(&ua, &a, 4); memcpy(&uc, &c, 4);
    if (ua != uc && !(isnan(a) && isnan(c))) ++bad;
  }
  printf("%llu\n", (unsigned long long)bad);
  return 0;
}
"""


def pin_glibc():
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "drv.c"), os.path.join(d, "drv")
        open(src, "w").write(DRIVER)
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-builtin", src,
                        os.path.join(ROOT, "oracle", "silu_ref.c"), "-lm", "-o", exe], check=True)
        return int(subprocess.run([exe], check=True, capture_output=True, text=True).stdout)


def pin_sleef():
    W = {"AVX512": 32, "AVX2": 16}[torch.backends.cpu.get_cpu_capability()]
    CH = 1 << 26
    bad = 0
    for c in range(1 << 6):
        x = np.arange(c * CH, (c + 1) * CH, dtype=np.uint64).astype(np.uint32).view(np.float32)
        want = torch.nn.functional.silu(torch.from_numpy(x)).numpy()
        got = O.silu_forward(x, (0, 1))   # W = 0: every element on the vectorized path
        nan = np.isnan(want) & np.isnan(got)
        bad += int(((want.view(np.uint32) != got.view(np.uint32)) & ~nan).sum())
    return bad


if __name__ == "__main__":
    t0 = time.time()
    print("glibc expf restatement vs libm expf, all 2^32 inputs: mismatches =", pin_glibc(),
          f"({time.time() - t0:.0f} s)", flush=True)
    t0 = time.time()
    print("vectorized silu restatement vs torch CPU F.silu, all 2^32 inputs: mismatches =", pin_sleef(),
          f"({time.time() - t0:.0f} s)", flush=True)
