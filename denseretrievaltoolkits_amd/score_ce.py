"""Fused in-batch score matrix + cross entropy with autograd, on the HIP kernels.

Forward   S = q @ p^T (exact-f32 MFMA), loss = scale * mean_i CE(S_i, i * stride)
Backward  dS = scale * g / m * (softmax(S) - onehot);  dq = dS @ p;  dp = dS^T @ q
Replaces ``torch.matmul(q_reps, p_reps.transpose(0, 1))`` + ``nn.CrossEntropyLoss``
in DRModel.forward (DRT/model/biencoder.py:107-119) and SimpleContrastiveLoss
(DRT/trainer/losses.py:11-17).
"""
from __future__ import annotations

import torch

from . import _native, ops


def _f32(t):
    return t.detach().to(torch.float32).contiguous()


def gemm_nt_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    lib = _native.load()
    m, k = a.shape
    n = b.shape[0]
    out = torch.empty((m, n), dtype=torch.float32, device=a.device)
    _native.check(lib.drt_gemm_nt_f32(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k, a.stride(0),
                                      b.stride(0), out.stride(0), _native.stream_ptr(a.device)), "drt_gemm_nt_f32")
    return out


def transpose_f32(x: torch.Tensor) -> torch.Tensor:
    lib = _native.load()
    r, c = x.shape
    y = torch.empty((c, r), dtype=torch.float32, device=x.device)
    _native.check(lib.drt_transpose_f32(x.data_ptr(), r, c, y.data_ptr(), _native.stream_ptr(x.device)),
                  "drt_transpose_f32")
    return y


def gemm_f32(a: torch.Tensor, b: torch.Tensor, a_kc: bool, b_kc: bool, m: int, n: int, k: int) -> torch.Tensor:
    """C[m, n] = sum_k A(m, k) B(k, n) on the exact-f32 MFMA; A is a [m][k] (a_kc) or [k][m]
    row-major tensor, B is [n][k] (b_kc) or [k][n].  Split-K (deterministic) when the
    64 x 64 output tiles alone cannot fill the chip."""
    lib = _native.load()
    out = torch.empty((m, n), dtype=torch.float32, device=a.device)
    tiles = -(-m // 64) * -(-n // 64)
    splits = max(1, min(-(-320 // tiles), k // 128))
    ws = torch.empty((splits, m, n), dtype=torch.float32, device=a.device) if splits > 1 else None
    _native.check(lib.drt_gemm_f32(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k, a.stride(0), b.stride(0),
                                   out.stride(0), int(a_kc), int(b_kc), splits,
                                   ws.data_ptr() if ws is not None else None, _native.stream_ptr(a.device)),
                  "drt_gemm_f32")
    return out


def score_ce(q: torch.Tensor, p: torch.Tensor, target_stride: int, scale: float = 1.0):
    """(loss, scores) for in-batch negatives with target_i = i * target_stride.

    ``torch.ops.drt.score_ce_fwd`` (two host calls per step: drt_score_ce_fwd = split-K GEMM ->
    split reduce + LSE -> fixed-order mean, and in the backward drt_score_ce_bwd = dS -> dq and
    dp GEMMs in one grid -> split reductions), autograd registered in ops.py.  bf16 inputs are
    promoted to fp32 (the reference computes the loss in fp32) and their gradients cast back."""
    if not (q.is_cuda and p.is_cuda):
        raise ValueError("score_ce runs on the GPU only (no CPU fallback)")
    if q.dim() != 2 or p.dim() != 2 or q.shape[1] != p.shape[1]:
        raise ValueError(f"q {tuple(q.shape)} and p {tuple(p.shape)} differ in dimension")
    loss, scores, _ = ops.load().score_ce_fwd(q.float(), p.float(), int(target_stride), float(scale))
    return loss, scores
