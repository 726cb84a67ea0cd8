"""Compile the HIP sources under agilerl_amd/csrc into agilerl_amd/lib/libagx.so
(gfx950 only).  In-tree so the built library travels with the repository
snapshot to the GPU box."""

from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(HERE, "lib", "obj")
LIB = os.path.join(LIBDIR, "libagx.so")
ARCH = "gfx950"
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
CFLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
    "-Wall", "-Wno-unused-function", "-I", os.path.join(HERE, "..", "include"),
]


def _needs(obj: str, src: str, deps: list[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src, *deps])


def _compile(src: str, deps: list[str]) -> str:
    obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
    if _needs(obj, src, deps):
        cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr}")
    return obj


def build(verbose: bool = False) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    deps = sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(HERE, "..", "include", "agx.h")]
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, deps), srcs))
    if not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(verbose=True)
