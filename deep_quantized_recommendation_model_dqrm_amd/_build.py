"""Build libdqrm.so (HIP, gfx950) in-tree with hipcc.

The shared library is the product: every hot-path op of this package goes through its
C ABI (``include/dqrm.h``). It is built in-tree so that it travels with the repository
snapshot to the GPU box and is the file the Python processes load.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC_DIR = os.path.join(PKG_DIR, "csrc")
SOURCES = [os.path.join(CSRC_DIR, f) for f in ("dqrm_kernels.hip", "dqrm_coalesce.hip", "dqrm_dense.hip",
                                                "dqrm_input.hip", "dqrm_sync.hip", "dqrm_exchange.hip", "dqrm_lookup.hip",
                                                "dqrm_comm.hip", "dqrm_apply.hip", "dqrm_apply_merge.hip")]
DEVICE_HEADER = os.path.join(CSRC_DIR, "dqrm_device.h")
HEADER = os.path.join(REPO_DIR, "include", "dqrm.h")
INTERNAL_HEADER = os.path.join(CSRC_DIR, "dqrm_internal.h")
LIB_PATH = os.path.join(PKG_DIR, "libdqrm.so")

HIPCC_FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-fPIC",
    # The reference's `1/s*x + 0`, `(g*s)/s` and `W + (-lr*v)` are separately rounded
    # operations; contraction would change bits. Intended FMAs are explicit fmaf().
    "-ffp-contract=off",
    "-Wall",
    "-Wno-unused-function",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libdqrm)")


def _obj(src: str) -> str:
    return os.path.splitext(src)[0] + ".o"


def _stale(out: str, deps) -> bool:
    return not os.path.exists(out) or any(os.path.getmtime(p) > os.path.getmtime(out) for p in deps)


def needs_build() -> bool:
    return _stale(LIB_PATH, [*SOURCES, HEADER, INTERNAL_HEADER, DEVICE_HEADER, __file__])


def build(force: bool = False, verbose: bool = True, relink: bool = False) -> str:
    """Compile csrc/*.hip (one object per translation unit, rebuilt when stale) and link
    libdqrm.so next to this file. relink: link even when nothing is stale."""
    if not force and not relink and not needs_build():
        return LIB_PATH
    objs, jobs = [], []
    for src in SOURCES:  # translation units compile in parallel (one hipcc each)
        obj = _obj(src)
        if force or _stale(obj, [src, HEADER, INTERNAL_HEADER, DEVICE_HEADER, __file__]):
            tmp = obj + ".tmp.o"
            cmd = [hipcc(), *HIPCC_FLAGS, "-I", os.path.join(REPO_DIR, "include"), "-c", src, "-o", tmp]
            if verbose:
                print("[dqrm] " + " ".join(cmd), file=sys.stderr)
            jobs.append((subprocess.Popen(cmd), cmd, tmp, obj))
        objs.append(obj)
    failed = None
    for proc, cmd, tmp, obj in jobs:
        if proc.wait() != 0:
            failed = failed or subprocess.CalledProcessError(proc.returncode, cmd)
        elif failed is None:
            os.replace(tmp, obj)
    if failed is not None:
        raise failed
    tmp = LIB_PATH + ".tmp"
    cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", tmp]
    if verbose:
        print("[dqrm] " + " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    build(force="--force" in sys.argv)
