"""Tensor-level wrappers over the C-ABI (``include/drt.h``).

Every function here launches a hand-written gfx950 kernel from
``libdrt_hip.so`` on torch's current HIP stream.  Inputs must be CUDA (HIP)
tensors; there is deliberately no CPU path — a missing extension or a CPU
tensor raises.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _native

_ws_cache: dict = {}


def _require_device(*ts: torch.Tensor) -> None:
    for t in ts:
        if not t.is_cuda:
            raise ValueError("DRT kernels run on the GPU only (got a CPU tensor; no CPU fallback exists)")


def _workspace(device: torch.device, nbytes: int) -> torch.Tensor:
    """Scratch buffer per (device, current stream): launches on different streams never share one."""
    key = (device.type, device.index, _native.stream_ptr(device))
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        _ws_cache[key] = buf
    return buf


def ip_topk_workspace_bytes(nq: int, n: int, d: int, k: int) -> int:
    return int(_native.load().drt_ip_topk_workspace(nq, n, d, k))


def ip_topk(q: torch.Tensor, p: torch.Tensor, k: int, id_offset: int = 0, resolve: bool = True,
            out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
            status: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Exact inner-product top-k of `q` [nq, d] against corpus shard `p` [n, d] (bf16).

    Returns (scores fp32 [nq, k], ids int64 [nq, k], status int32 [nq]) ordered by
    (score desc, id asc); ids are ``id_offset + row``.  With ``resolve`` the
    (rare) uncertified queries are recomputed exactly before returning (this
    synchronises the stream); without it the caller must inspect ``status``.
    """
    lib = _native.load()
    _require_device(q, p)
    if q.dtype != torch.bfloat16 or p.dtype != torch.bfloat16:
        raise ValueError("ip_topk expects bf16 queries and corpus")
    if q.dim() != 2 or p.dim() != 2 or q.shape[1] != p.shape[1]:
        raise ValueError(f"shape mismatch: q {tuple(q.shape)} vs p {tuple(p.shape)}")
    q = q.contiguous()
    p = p.contiguous()
    nq, d = q.shape
    n = p.shape[0]
    dev = q.device
    if out is None:
        scores = torch.empty((nq, k), dtype=torch.float32, device=dev)
        ids = torch.empty((nq, k), dtype=torch.int64, device=dev)
    else:
        scores, ids = out
    if status is None:
        status = torch.empty((nq,), dtype=torch.int32, device=dev)
    wsb = lib.drt_ip_topk_workspace(nq, n, d, k)
    if wsb == 0 and nq > 0:
        raise ValueError(f"unsupported ip_topk shape nq={nq} n={n} d={d} k={k} (d % 64 == 0, d <= 1024, 1 <= k <= 2048)")
    ws = _workspace(dev, wsb)
    s = _native.stream_ptr(dev)
    _native.check(lib.drt_ip_topk_bf16(q.data_ptr(), nq, p.data_ptr() if n else None, n, d, k, id_offset,
                                       scores.data_ptr(), ids.data_ptr(), status.data_ptr(), ws.data_ptr(),
                                       wsb, s), "drt_ip_topk_bf16")
    if resolve:
        resolve_failed(q, p, k, id_offset, scores, ids, status)
    return scores, ids, status


def resolve_failed(q, p, k, id_offset, scores, ids, status) -> int:
    """Exact dense rescan of every query whose status is non-zero (synchronous)."""
    lib = _native.load()
    nres = _native.c_i64(0)
    nq, d = q.shape
    n = p.shape[0]
    _native.check(lib.drt_ip_topk_resolve(q.data_ptr(), nq, p.data_ptr() if n else None, n, d, k, id_offset,
                                          scores.data_ptr(), ids.data_ptr(), status.data_ptr(),
                                          _native.ctypes.byref(nres), _native.stream_ptr(q.device)),
                  "drt_ip_topk_resolve")
    return int(nres.value)


def topk_merge(scores: torch.Tensor, ids: torch.Tensor, k_out: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Merge per-shard lists [nparts, nq, k_in] (each sorted) into the global top-k_out."""
    lib = _native.load()
    _require_device(scores, ids)
    if scores.dim() != 3 or scores.shape != ids.shape:
        raise ValueError("topk_merge expects [nparts, nq, k] scores and ids")
    scores = scores.contiguous().float()
    ids = ids.contiguous().long()
    nparts, nq, k_in = scores.shape
    out_s = torch.empty((nq, k_out), dtype=torch.float32, device=scores.device)
    out_i = torch.empty((nq, k_out), dtype=torch.int64, device=scores.device)
    _native.check(lib.drt_topk_merge(scores.data_ptr(), ids.data_ptr(), nq, nparts, k_in, k_out,
                                     out_s.data_ptr(), out_i.data_ptr(), _native.stream_ptr(scores.device)),
                  "drt_topk_merge")
    return out_s, out_i


# ---------------------------------------------------------------------------
# Global-threshold distributed search (include/drt.h, drt_ip_topk_dist_*)
# ---------------------------------------------------------------------------
def sample_rank(k: int) -> int:
    r = int(_native.load().drt_ip_topk_sample_rank(k))
    if r <= 0:
        raise ValueError(f"unsupported k={k}")
    return r


def _dist_ws(q, n_local, n_global, k):
    lib = _native.load()
    nq, d = q.shape
    wsb = lib.drt_ip_topk_dist_workspace(nq, n_local, n_global, d, k)
    if wsb == 0 and nq > 0:
        raise ValueError(f"unsupported dist shape nq={nq} n_local={n_local} n_global={n_global} d={d} k={k}")
    return _workspace(q.device, wsb), wsb


def dist_sample(q: torch.Tensor, p: torch.Tensor, n_global: int, k: int) -> torch.Tensor:
    """Best r sampled score keys of this shard, [nq, r] int32 (uint32 bit patterns, ascending)."""
    lib = _native.load()
    _require_device(q, p)
    q = q.contiguous()
    p = p.contiguous()
    nq, d = q.shape
    best = torch.empty((nq, sample_rank(k)), dtype=torch.int32, device=q.device)
    ws, wsb = _dist_ws(q, p.shape[0], n_global, k)
    _native.check(lib.drt_ip_topk_dist_sample(q.data_ptr(), nq, p.data_ptr() if p.shape[0] else None, p.shape[0],
                                              n_global, d, k, best.data_ptr(), ws.data_ptr(), wsb,
                                              _native.stream_ptr(q.device)), "drt_ip_topk_dist_sample")
    return best


def dist_tau(lists: torch.Tensor, k: int) -> torch.Tensor:
    """Global threshold from all shards' lists [nlists, nq, r] -> tau [nq] fp32."""
    lib = _native.load()
    _require_device(lists)
    lists = lists.contiguous()
    nlists, nq, _ = lists.shape
    tau = torch.empty((nq,), dtype=torch.float32, device=lists.device)
    _native.check(lib.drt_ip_topk_dist_tau(lists.data_ptr(), nq, nlists, k, tau.data_ptr(),
                                           _native.stream_ptr(lists.device)), "drt_ip_topk_dist_tau")
    return tau


def dist_filter(q: torch.Tensor, p: torch.Tensor, n_global: int, k: int, id_offset: int,
                tau: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """This shard's packed top-k of rows scoring >= tau: [nq, k + 1] int64 (uint64 bit patterns)."""
    lib = _native.load()
    _require_device(q, p, tau)
    q = q.contiguous()
    p = p.contiguous()
    nq, d = q.shape
    if out is None:
        out = torch.empty((nq, k + 1), dtype=torch.int64, device=q.device)
    ws, wsb = _dist_ws(q, p.shape[0], n_global, k)
    _native.check(lib.drt_ip_topk_dist_filter(q.data_ptr(), nq, p.data_ptr() if p.shape[0] else None, p.shape[0],
                                              n_global, d, k, id_offset, tau.data_ptr(), out.data_ptr(),
                                              ws.data_ptr(), wsb, _native.stream_ptr(q.device)),
                  "drt_ip_topk_dist_filter")
    return out


def merge_packed(parts: torch.Tensor, k: int, n_global: int):
    """[nparts, nq, k + 1] packed lists -> (scores [nq,k], ids [nq,k], status [nq] int32; 0 = exact)."""
    lib = _native.load()
    _require_device(parts)
    parts = parts.contiguous()
    nparts, nq, kp1 = parts.shape
    if kp1 != k + 1:
        raise ValueError("merge_packed expects [nparts, nq, k + 1]")
    dev = parts.device
    s = torch.empty((nq, k), dtype=torch.float32, device=dev)
    i = torch.empty((nq, k), dtype=torch.int64, device=dev)
    st = torch.empty((nq,), dtype=torch.int32, device=dev)
    _native.check(lib.drt_topk_merge_packed(parts.data_ptr(), nq, nparts, k, n_global, s.data_ptr(), i.data_ptr(),
                                            st.data_ptr(), _native.stream_ptr(dev)), "drt_topk_merge_packed")
    return s, i, st


def gemm_nt_f32(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """C = a @ b.T with bf16 inputs and fp32 accumulation/output (MFMA)."""
    lib = _native.load()
    _require_device(a, b)
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise ValueError("gemm_nt_f32 expects bf16 operands")
    a = a.contiguous()
    b = b.contiguous()
    m, d = a.shape
    n = b.shape[0]
    if out is None:
        out = torch.empty((m, n), dtype=torch.float32, device=a.device)
    _native.check(lib.drt_gemm_nt_bf16_f32(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, d, out.stride(0),
                                           _native.stream_ptr(a.device)), "drt_gemm_nt_bf16_f32")
    return out
