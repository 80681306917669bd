"""Build the in-tree HIP shared library (gfx950) — `python -m vsiquantization_amd._build`.

The kernels are split over a few translation units (csrc/*.hip) that hipcc
compiles in parallel to objects under build/, then links into `_vsiq_hip.so`
next to this file, so the built library travels with the repository snapshot to
the GPU box.
Flags that matter for parity with the reference's CPU arithmetic:
  -ffp-contract=off                       no FMA contraction of (q - zp) * s etc.
  -fhip-fp32-correctly-rounded-divide-sqrt   IEEE x / s
  -fno-gpu-flush-denormals-to-zero        keep fp32 denormals (torch CPU keeps them)
  -mcode-object-version=5                 loadable by torch's bundled ROCm 7.0 runtime
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJDIR = os.path.join(ROOT, "build", "vsiq")
OUT = os.path.join(HERE, "_vsiq_hip.so")
TORCH_EXT_SRC = os.path.join(CSRC, "torch_ops.cpp")
TORCH_EXT_OUT = os.path.join(HERE, "_vsiq_torch.so")
ARCH = os.environ.get("VSIQ_OFFLOAD_ARCH", "gfx950")

FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-ffp-contract=off",
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-fno-gpu-flush-denormals-to-zero",
    "-mcode-object-version=5",
    "-Wall",
]


# per-source extra flags.  k_flat.hip (K2 / K2p / K2m observers): without SLP
# vectorization the observer's |x| sums stay scalar adds with free abs modifiers instead
# of v_pk_add_f32 fed by v_and / v_mov pairs -- C5's K2m 175 -> 168 us on MI355X (C2 / C3
# / C4 kernels measured unchanged with it, so they keep the default)
FILE_FLAGS = {"k_flat.hip": ["-fno-slp-vectorize"]}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build vsiquantization_amd)")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def host_sources():
    """Host-only C++ (csrc/host_*.cpp: the CPU-tensor path's AVX-512 loops), compiled by
    the system C++ compiler; torch_ops.cpp is the separate torch extension."""
    return sorted(glob.glob(os.path.join(CSRC, "host_*.cpp")))


HOST_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall"]


def cxx() -> str:
    for cand in (os.environ.get("CXX"), shutil.which("g++"), shutil.which("c++")):
        if cand and os.path.exists(cand):
            return cand
    return hipcc()


def _deps():
    return (sources() + host_sources() + glob.glob(os.path.join(CSRC, "*.cuh")) + glob.glob(os.path.join(CSRC, "*.h"))
            + [os.path.join(ROOT, "include", "vsiq.h"), os.path.abspath(__file__)])


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in _deps() if os.path.exists(d))


def build(force: bool = False, verbose: bool = True, jobs: int = 0) -> str:
    if not force and not needs_build():
        return OUT
    os.makedirs(OBJDIR, exist_ok=True)
    cc = hipcc()
    inc = ["-I", os.path.join(ROOT, "include"), "-I", CSRC]
    newest_dep = max(os.path.getmtime(d) for d in _deps() if d.endswith((".cuh", ".h", ".py")))

    def compile_one(src):
        obj = os.path.join(OBJDIR, os.path.splitext(os.path.basename(src))[0] + ".o")
        if (not force and os.path.exists(obj) and os.path.getmtime(obj) > os.path.getmtime(src)
                and os.path.getmtime(obj) > newest_dep):
            return obj
        if src.endswith(".cpp"):
            cmd = [cxx(), *HOST_FLAGS, *inc, "-c", "-o", obj + ".tmp", src]
        else:
            cmd = [cc, *FLAGS, *FILE_FLAGS.get(os.path.basename(src), []), *inc, "-c", "-o", obj + ".tmp", src]
        if verbose:
            print("[vsiq build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
        return obj

    jobs = jobs or min(16, os.cpu_count() or 4)
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, sources() + host_sources()))
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT + ".tmp", *objs]
    if verbose:
        print("[vsiq build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


def needs_torch_ext_build() -> bool:
    if not os.path.exists(TORCH_EXT_OUT):
        return True
    t = os.path.getmtime(TORCH_EXT_OUT)
    deps = [TORCH_EXT_SRC, OUT, os.path.join(ROOT, "include", "vsiq.h"), os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_torch_ext(force: bool = False, verbose: bool = True) -> str:
    """`_vsiq_torch.so`: the C++ autograd nodes of csrc/torch_ops.cpp (pybind11 module
    against torch's headers, host code only), linked to `_vsiq_hip.so` ($ORIGIN rpath)
    and to torch's own libraries (so the HIP runtime is torch's)."""
    if not force and not needs_torch_ext_build():
        return TORCH_EXT_OUT
    import sysconfig

    import torch
    import torch.utils.cpp_extension as ce
    inc = ce.include_paths(device_type="cuda") + [sysconfig.get_paths()["include"],
                                                   os.path.join(ROOT, "include")]
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    cmd = [hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
           "-DTORCH_EXTENSION_NAME=_vsiq_torch", "-Wno-unused-result", "-Wno-deprecated-declarations",
           *[f"-I{i}" for i in inc], TORCH_EXT_SRC, "-o", TORCH_EXT_OUT + ".tmp",
           f"-L{tlib}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
           f"-L{HERE}", "-l:_vsiq_hip.so", f"-Wl,-rpath,{tlib}", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print("[vsiq build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(TORCH_EXT_OUT + ".tmp", TORCH_EXT_OUT)
    return TORCH_EXT_OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_torch_ext(force="--force" in sys.argv)
