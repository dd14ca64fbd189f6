"""CPU-side checks of the C-ABI boundary (no GPU compute)."""
import ctypes
import os
import re

from conftest import REPO


def _declared_symbols():
    hdr = open(os.path.join(REPO, "include", "drt.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    names = re.findall(r"\b(drt_[a-z0-9_]+)\s*\(", hdr)
    return sorted(set(names))


def test_library_builds_and_exports_every_declared_symbol():
    from denseretrievaltoolkits_amd import build_native, _native
    path = build_native.build()
    assert os.path.exists(path)
    lib = ctypes.CDLL(path)
    declared = _declared_symbols()
    assert "drt_ip_topk_bf16" in declared and "drt_topk_merge" in declared
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in include/drt.h but not exported"
    # the ctypes binding covers exactly the declared surface
    assert sorted(_native.EXPORTED) == declared


def test_host_only_entry_points():
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    assert b"gfx950" in lib.drt_version()
    # workspace query is pure host arithmetic
    ws = lib.drt_ip_topk_workspace(128, 10_000_000, 768, 1000)
    assert ws > 0
    # unsupported shapes are rejected with 0
    assert lib.drt_ip_topk_workspace(128, 1000, 100, 10) == 0      # d % 64 != 0
    assert lib.drt_ip_topk_workspace(128, 1000, 768, 4096) == 0    # k > 2048


def test_invalid_arguments_rejected_without_gpu():
    from denseretrievaltoolkits_amd import _native
    lib = _native.load()
    # DRT_EINVAL is returned before any HIP call for bad shapes
    rc = lib.drt_ip_topk_bf16(None, 4, None, 10, 100, 5, 0, None, None, None, None, 0, None)
    assert rc == _native.DRT_EINVAL
    rc = lib.drt_topk_merge(None, None, 4, 0, 10, 10, None, None, None)
    assert rc == _native.DRT_EINVAL
    rc = lib.drt_gemm_nt_bf16_f32(None, None, None, 4, 4, 100, 4, None)
    assert rc == _native.DRT_EINVAL
