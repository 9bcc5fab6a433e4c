"""Builds librpgpu.so in-tree: hand-written gfx950 kernels + the C-ABI host
runtime (hipcc), linked into one shared library.

No JIT, no torch extension: the .so lives next to this file so it travels to
the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INC = os.path.join(ROOT, "include")
OUT = os.path.join(HERE, "librpgpu.so")
BUILD = os.path.join(HERE, "_build")
ARCH = os.environ.get("RPGPU_ARCH", "gfx950")

HIP_SOURCES = ["rp_kernels.hip", "rp_validate.hip", "rp_codec.hip", "rp_inflate.hip", "rp_compress.hip", "rp_index.hip", "rp_runtime.hip"]
CXX_SOURCES = ["rp_hostcodec.cpp"]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {cmd[0]} ({r.returncode})")
    return r


def _stale(obj, srcs):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(s) > t for s in srcs)


VARIANTS = {
    # name: (library, build dir, extra flags)
    "": (OUT, BUILD, []),
    "checked": (os.path.join(HERE, "librpgpu_checked.so"), BUILD + "_checked", ["-DRPGPU_CHECKED"]),
    "stamps": (os.path.join(HERE, "librpgpu_stamps.so"), BUILD + "_stamps", ["-DRPGPU_STAMPS"]),
    # environment overrides (RPGPU_DEBUG_SYNC, RPGPU_POOL_SLABS, ...): diagnostics only
    "diag": (os.path.join(HERE, "librpgpu_diag.so"), BUILD + "_diag", ["-DRPGPU_DIAG"]),
}


def build(force: bool = False, verbose: bool = False, checked: bool = False, variant: str = "") -> str:
    """checked=True builds librpgpu_checked.so (bounds-checked kernels);
    variant="stamps" builds librpgpu_stamps.so (per-phase cycle stamps)."""
    if checked:
        variant = "checked"
    out, bdir, extra = VARIANTS[variant]
    os.makedirs(bdir, exist_ok=True)
    hipcc = _hipcc()
    headers = [os.path.join(INC, "rpgpu.h"), os.path.join(CSRC, "rp_internal.h"), os.path.join(CSRC, "rp_device.h"),
               os.path.join(CSRC, "rp_zstd_core.h")]
    objs, cmds = [], []
    for src in HIP_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(bdir, src + ".o")
        if force or _stale(o, [s] + headers):
            cmds.append([hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-I", INC, "-I", CSRC,
                         "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-label"] + extra
                        + ["-c", s, "-o", o])
        objs.append(o)
    for src in CXX_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(bdir, src + ".o")
        if force or _stale(o, [s] + headers):
            cmds.append(["g++", "-O2", "-fPIC", "-std=c++17", "-I", INC, "-Wall"] + extra + ["-c", s, "-o", o])
        objs.append(o)
    if verbose:
        for cmd in cmds:
            print(" ".join(cmd))
    # one compiler per source, in parallel (each hipcc is single-threaded)
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 1), 8))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(_run, cmds))
    if force or _stale(out, objs):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + ["-ldl", "-lpthread"]
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
    return out


SURFACES_SRC = os.path.join(ROOT, "tests", "cpp", "surfaces_main.cpp")
SURFACES_BIN = os.path.join(ROOT, "tests", "cpp", "_bin", "surfaces_test")


def build_surfaces_test(force: bool = False) -> str:
    """Host-only driver of include/rpgpu_redpanda.h (the C++ drop-in
    surfaces), linked against librpgpu.so by a relative runpath so the built
    binary travels with the tree."""
    lib = build()
    hdrs = [os.path.join(INC, "rpgpu.h"), os.path.join(INC, "rpgpu_redpanda.h")]
    if force or _stale(SURFACES_BIN, [SURFACES_SRC, lib] + hdrs):
        os.makedirs(os.path.dirname(SURFACES_BIN), exist_ok=True)
        _run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-I", INC, SURFACES_SRC, "-o", SURFACES_BIN, "-L", HERE, "-l:librpgpu.so",
              "-Wl,-rpath,$ORIGIN/../../../redpanda_amd"])
    return SURFACES_BIN


ZSHOST_SRC = os.path.join(ROOT, "tests", "cpp", "zstd_core_host.cpp")
ZSHOST_LIB = os.path.join(ROOT, "tests", "cpp", "_bin", "libzshost.so")


def build_zstd_host(force: bool = False) -> str:
    """rp_zstd_core.h built for the host (test infrastructure: the GPU tests
    compare the device decoder with the same logic on the host)."""
    hdr = os.path.join(CSRC, "rp_zstd_core.h")
    if force or _stale(ZSHOST_LIB, [ZSHOST_SRC, hdr]):
        os.makedirs(os.path.dirname(ZSHOST_LIB), exist_ok=True)
        _run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", ZSHOST_LIB, ZSHOST_SRC])
    return ZSHOST_LIB


if __name__ == "__main__":
    v = "checked" if "--checked" in sys.argv else "stamps" if "--stamps" in sys.argv else \
        "diag" if "--diag" in sys.argv else ""
    print(build(force="--force" in sys.argv, verbose=True, variant=v))
