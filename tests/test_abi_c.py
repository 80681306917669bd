"""The C ABI from plain C (no Python, no torch): include/vsiq.h compiles as C99 and a C
program links _vsiq_hip.so and calls the host-side entry points (version, error
strings, sizes, argument validation) -- what a non-Python host binding relies on
(INTEGRATION.md §2).  No GPU: nothing here launches a kernel."""
import os
import shutil
import subprocess

import pytest

from vsiquantization_amd import _build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

C_SRC = r"""
#include <stdio.h>
#include <string.h>
#include "vsiq.h"

int main(void) {
  if (vsiq_abi_version() != VSIQ_ABI_VERSION) return 1;
  if (strcmp(vsiq_error_string(0), "success") != 0) return 2;
  if (vsiq_mask_words(2, 257) != 2 * 4 * 2) return 3;                 /* 4 words per 256 elements */
  if (vsiq_mask_words(-1, 4) >= 0) return 4;
  if (vsiq_fq_fwd_f32(NULL, NULL, NULL, NULL, -1, NULL, NULL, 1.0, NULL, 0.0, 0, 0, 0, 1, NULL) != VSIQ_E_ARG)
    return 5;                                                           /* n < 0 */
  if (vsiq_fq_fwd_f32(NULL, NULL, NULL, NULL, 0, NULL, NULL, 1.0, NULL, 0.0, 0, 0, 0, 1, NULL) != 0)
    return 6;                                                           /* n == 0: no-op */
  if (vsiq_set_tuning(VSIQ_TUNE_XCD_ORDER, 3) == 0) return 7;
  if (vsiq_observe_part_records(1) != 4) return 8;                    /* one record per wave */
  if (vsiq_lsq_fold_multi(NULL, 0, NULL) != 0) return 9;
  printf("ok %d\n", vsiq_abi_version());
  return 0;
}
"""


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no C compiler")
def test_header_is_c99_and_links_from_c(tmp_path):
    assert os.path.exists(_build.OUT), "run __graft_entry__.build() first"
    src = tmp_path / "abi.c"
    src.write_text(C_SRC)
    exe = tmp_path / "abi"
    libdir = os.path.dirname(_build.OUT)
    lib = os.path.basename(_build.OUT)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I", os.path.join(ROOT, "include"),
                    str(src), "-o", str(exe), f"-L{libdir}", f"-l:{lib}", f"-Wl,-rpath,{libdir}"],
                   check=True, capture_output=True, text=True)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, (p.returncode, p.stdout, p.stderr)
    assert p.stdout.startswith("ok ")
