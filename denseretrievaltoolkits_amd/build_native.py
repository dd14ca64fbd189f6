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
OPS_LIB_PATH = os.path.join(PKG_DIR, "_drt_ops.so")
OPS_SRC = os.path.join(CSRC, "torch_ops.cpp")
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
        # SONAME: the custom-op library links libdrt_hip.so by that name, and the dynamic loader
        # then reuses the copy _native.py already loaded (one set of globals: profiling, switches)
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Wl,-soname,libdrt_hip.so", *objs, "-o", tmp]
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"link failed:\n{p.stderr}")
        os.replace(tmp, LIB_PATH)
    build_ops(force=force, verbose=verbose)
    return LIB_PATH


def build_ops(force: bool = False, verbose: bool = False) -> str:
    """torch.ops.drt.* (csrc/torch_ops.cpp): host-only C++ against torch's headers, linked to
    libdrt_hip.so (rpath $ORIGIN) and torch's libraries."""
    deps = [OPS_SRC, LIB_PATH] + _headers()
    if not force and not _stale(OPS_LIB_PATH, deps):
        return OPS_LIB_PATH
    import torch
    from torch.utils import cpp_extension as ce
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        raise RuntimeError("no host C++ compiler for the torch custom-op library")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    inc = [f"-I{p}" for p in ce.include_paths()] + ["-I/opt/rocm/include", f"-I{os.path.join(REPO_DIR, 'include')}"]
    libdirs = ce.library_paths()
    tmp = OPS_LIB_PATH + ".tmp"
    cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1",
           "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_drt_ops", *inc, OPS_SRC, "-o", tmp,
           *[f"-L{d}" for d in libdirs], "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch", f"-L{PKG_DIR}", "-ldrt_hip",
           "-Wl,-rpath,$ORIGIN", "-Wl,--no-as-needed"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"torch ops build failed:\n{p.stderr[-4000:]}")
    os.replace(tmp, OPS_LIB_PATH)
    return OPS_LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
