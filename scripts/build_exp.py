"""Build experiment variants of librpgpu.so: redpanda_amd/librpgpu_<name>.so
with an alternate kernel source (--unit, default rp_validate.hip) and/or extra defines; the other objects
come from the main build.  Usage:
  python scripts/build_exp.py NAME [--src path/to/rp_validate.hip] [--unit rp_codec.hip] [--base diag] [-DFOO ...]
Load with RPGPU_VARIANT=NAME.  Diagnostics only, never the product."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from redpanda_amd import build as B  # noqa: E402

name = sys.argv[1]
args = sys.argv[2:]
unit = "rp_validate.hip"
if "--unit" in args:  # which translation unit gets the source / defines
    i = args.index("--unit")
    unit = args[i + 1]
    del args[i:i + 2]
src = os.path.join(B.CSRC, unit)
if "--src" in args:
    i = args.index("--src")
    src = os.path.abspath(args[i + 1])
    del args[i:i + 2]
base = ""
if "--base" in args:  # the variant whose other objects are linked (e.g. diag)
    i = args.index("--base")
    base = args[i + 1]
    del args[i:i + 2]
defs = [a for a in args if a.startswith("-D")]
B.build(variant=base)
bdir = os.path.join(B.HERE, "_build_exp_" + name)
os.makedirs(bdir, exist_ok=True)
obj = os.path.join(bdir, unit + ".o")
B._run([B._hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-fPIC", "-std=c++17", "-I", B.INC, "-I", B.CSRC,
        "-Wno-unused-function", "-Wno-unused-variable"] + defs + ["-c", src, "-o", obj])
bbuild = B.VARIANTS[base][1]
objs = [os.path.join(bbuild, s + ".o") for s in B.HIP_SOURCES + B.CXX_SOURCES if s != unit] + [obj]
out = os.path.join(B.HERE, f"librpgpu_{name}.so")
B._run([B._hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", out] + objs + ["-ldl", "-lpthread"])
print(out)
