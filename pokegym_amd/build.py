"""Build the HIP extension (gfx950) in-tree: pokegym_amd/lib/libpokegym_amd.so.

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build container and the
resulting .so travels to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libpokegym_amd.so")
SOURCES = ["pk_step.hip", "pk_kernels.hip", "pk_reward.hip", "pk_capi.cpp"]
HEADERS = ["pk_layout.h", "pk_ucode.h", "pk_render.h", "pk_reward.h", "pk_reward_tables.h", os.path.join("..", "..", "include", "pokegym_amd.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PK_OFFLOAD_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, out: str | None = None, extra: list | None = None) -> str:
    """Compile the gfx950 library; `out`/`extra` build an alternative copy for A/B experiments."""
    lib = out or LIB
    if out is None and not force and not _stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    objs = []
    # (source, object stem, extra defines): K1 is compiled twice, the default kernel and the
    # small-LDS kernel for concurrent sub-batch ranges (pk_layout.h PK_K1_SMALL)
    units = [(src, os.path.splitext(src)[0], []) for src in SOURCES] + [("pk_step.hip", "pk_step_small", ["-DPK_K1_SMALL"])]
    for src, stem, defs in units:
        obj = os.path.join(LIBDIR, stem + (".alt.o" if out else ".o"))
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
               "-Wno-unused-function", "-Wno-bitwise-instead-of-logical", "-c", "-o", obj] + defs + list(extra or [])
        if src.endswith(".cpp"):
            cmd += ["-x", "hip"]
        cmd.append(os.path.join(CSRC, src))
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = lib + ".tmp"
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs, check=True)
    os.replace(tmp, lib)
    for o in objs:
        os.remove(o)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
