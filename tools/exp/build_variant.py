"""Build a variant of the product library with extra -D flags (experiments only).
usage: python tools/exp/build_variant.py OUT.so -DNAME=VALUE ..."""
import glob, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vsiquantization_amd import _build  # noqa
out, defs = sys.argv[1], sys.argv[2:]
tmp = os.path.join(ROOT, "build", "variant_" + os.path.basename(out).replace(".so", ""))
os.makedirs(tmp, exist_ok=True)
inc = ["-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "vsiquantization_amd", "csrc")]
objs = []
srcs = sorted(glob.glob(os.path.join(ROOT, "vsiquantization_amd", "csrc", "*.hip")))
procs = []
for src in srcs:
    obj = os.path.join(tmp, os.path.basename(src) + ".o")
    objs.append(obj)
    procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc", *_build.FLAGS, *_build.FILE_FLAGS.get(os.path.basename(src), []),
                                   *defs, *inc, "-c", "-o", obj, src]))
for src in _build.host_sources():   # the CPU-tensor path's host loops (g++)
    obj = os.path.join(tmp, os.path.basename(src) + ".o")
    objs.append(obj)
    procs.append(subprocess.Popen([_build.cxx(), *_build.HOST_FLAGS, *inc, "-c", "-o", obj, src]))
assert all(p.wait() == 0 for p in procs)
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs])
print("built", out)
