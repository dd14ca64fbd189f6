"""In-tree build of the HIP extension ``libdrt_hip.so`` for gfx950.

The library is a plain C-ABI shared object (``include/drt.h``); Python reaches it
through ctypes (``_native.py``).  Built in-tree so the ``.so`` travels to the GPU
box with the repository snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(PKG_DIR, "build")
LIB_PATH = os.path.join(PKG_DIR, "libdrt_hip.so")
ARCH = "gfx950"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the DRT HIP extension cannot be built")


def sources() -> list[str]:
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers() -> list[str]:
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(REPO_DIR, "include", "drt.h"))
    return hs


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, jobs: int = 8) -> str:
    """Compile every csrc/*.hip for gfx950 and link libdrt_hip.so. Returns its path."""
    os.makedirs(BUILD_DIR, exist_ok=True)
    hipcc = _hipcc()
    srcs = sources()
    hdrs = _headers()
    flags = [
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-Wno-unused-result",
        "-Wno-unused-value",
        f"-I{os.path.join(REPO_DIR, 'include')}",
    ]
    objs = []
    todo = []
    for src in srcs:
        obj = os.path.join(BUILD_DIR, os.path.basename(src)[:-4] + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            todo.append((src, obj))

    def _compile(so):
        src, obj = so
        cmd = [hipcc, *flags, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{p.stderr}")
        return obj

    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            list(ex.map(_compile, todo))
    if force or todo or _stale(LIB_PATH, objs):
        tmp = LIB_PATH + ".tmp"
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp]
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"link failed:\n{p.stderr}")
        os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
