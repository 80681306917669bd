"""Child of tests/test_host_simd.py: runs the host loops (vsiq_host_*) on the shared
inputs and saves every output; VSIQ_HOST_SIMD=0 in the environment selects the scalar
loops (read once per process)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.host_simd_cases import cases, run_case  # noqa: E402


def main():
    out = {}
    for name, args in cases().items():
        for k, v in run_case(*args).items():
            out[f"{name}.{k}"] = v
    np.savez(sys.argv[1], **out)


if __name__ == "__main__":
    torch.set_num_threads(1)
    main()
