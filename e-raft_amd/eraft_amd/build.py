"""Compile libcorr_mi355x.so (the gfx950 HIP kernels + C-ABI) in-tree with hipcc.

The .so lands in ``e-raft_amd/eraft_amd/_build/`` (git-ignored, but it travels to the GPU
box with the gpurun snapshot).  No JIT cache, no torch C++ extension: the boundary is the
plain C-ABI of include/corr_mi355x.h, loaded with ctypes.
"""
from __future__ import annotations

import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(os.path.dirname(PKG), "csrc")
OUT_DIR = os.path.join(PKG, "_build")
SO_NAME = "libcorr_mi355x.so"
SO_PATH = os.path.join(OUT_DIR, SO_NAME)
SOURCES = ["corr_build.hip", "corr_build_split.hip", "corr_build_bf16.hip", "corr_lookup.hip", "corr_bwd.hip", "corr_bwd_split.hip", "corr_splat.hip",
           "corr_upsample.hip", "corr_voxel.hip",
           "corr_api.cpp"]
HEADERS = ["corr_common.h", "corr_build_common.h", os.path.join("..", "..", "include", "corr_mi355x.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -ffp-contract=off: the lookup / pool arithmetic is specified op-by-op (each fp32 op rounds
# once, fmaf only where the reference's ATen kernel fuses); the compiler must not contract.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC", "-shared", "-ffp-contract=off",
         "-Wall"]


def _stale() -> bool:
    if not os.path.exists(SO_PATH):
        return True
    t = os.path.getmtime(SO_PATH)
    deps = [os.path.join(SRC, s) for s in SOURCES + HEADERS] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps)


OBJ_DIR = os.path.join(OUT_DIR, "obj")


def _compile(src: str, force: bool, verbose: bool) -> str:
    """One translation unit -> _build/obj/<name>.o, rebuilt when it or a shared header is newer."""
    obj = os.path.join(OBJ_DIR, os.path.splitext(src)[0] + ".o")
    deps = [os.path.join(SRC, src)] + [os.path.join(SRC, h) for h in HEADERS] + [__file__]
    if not force and os.path.exists(obj) and all(os.path.getmtime(d) <= os.path.getmtime(obj) for d in deps):
        return obj
    flags = [f for f in FLAGS if f != "-shared"]
    cmd = [HIPCC, *flags, "-c", "-o", obj + ".tmp", os.path.join(SRC, src)]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(obj + ".tmp", obj)
    return obj


def build_library(force: bool = False, verbose: bool = False, jobs: int | None = None) -> str:
    """Build the shared library if any source is newer than it (translation units compiled in
    parallel, only the stale ones).  Returns its path."""
    if not force and not _stale():
        return SO_PATH
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(OBJ_DIR, exist_ok=True)
    jobs = jobs or min(len(SOURCES), int(os.environ.get("MAX_JOBS") or 0) or os.cpu_count() or 4, 16)
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, verbose), SOURCES))
    tmp = SO_PATH + ".tmp"
    cmd = [HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", tmp, *objs]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, SO_PATH)
    return SO_PATH


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
