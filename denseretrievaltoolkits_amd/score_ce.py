"""Fused in-batch score matrix + cross entropy with autograd, on the HIP kernels.

Forward   S = q @ p^T (exact-f32 MFMA), loss = scale * mean_i CE(S_i, i * stride)
Backward  dS = scale * g / m * (softmax(S) - onehot);  dq = dS @ p;  dp = dS^T @ q
Replaces ``torch.matmul(q_reps, p_reps.transpose(0, 1))`` + ``nn.CrossEntropyLoss``
in DRModel.forward (DRT/model/biencoder.py:107-119) and SimpleContrastiveLoss
(DRT/trainer/losses.py:11-17).
"""
from __future__ import annotations

import torch

from . import _native


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


_WS = {}


def _workspace(lib, m: int, n: int, d: int, device) -> torch.Tensor:
    """Scratch of drt_score_ce_workspace bytes, cached per (device, shape): the training
    step reuses one buffer instead of allocating split-K partials on every call."""
    key = (device, m, n, d)
    ws = _WS.get(key)
    if ws is None:
        nbytes = int(lib.drt_score_ce_workspace(m, n, d))
        ws = torch.empty(max(1, (nbytes + 3) // 4), dtype=torch.float32, device=device)
        if len(_WS) > 8:
            _WS.clear()
        _WS[key] = ws
    return ws


class ScoreCE(torch.autograd.Function):
    """Two host calls per step: drt_score_ce_fwd (GEMM -> split reduce + LSE -> mean) and
    drt_score_ce_bwd (dS -> dq and dp GEMMs in one grid -> split reductions)."""

    @staticmethod
    def forward(ctx, q, p, target_stride: int, scale: float):
        if not (q.is_cuda and p.is_cuda):
            raise ValueError("ScoreCE runs on the GPU only (no CPU fallback)")
        lib = _native.load()
        qf, pf = _f32(q), _f32(p)
        m, d = qf.shape
        n = pf.shape[0]
        if pf.shape[1] != d:
            raise ValueError(f"q {tuple(qf.shape)} and p {tuple(pf.shape)} differ in dimension")
        dev = qf.device
        S = torch.empty((m, n), dtype=torch.float32, device=dev)
        lse = torch.empty(m, dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        ws = _workspace(lib, m, n, d, dev)
        _native.check(lib.drt_score_ce_fwd(qf.data_ptr(), pf.data_ptr(), m, n, d, int(target_stride), float(scale),
                                           S.data_ptr(), lse.data_ptr(), loss.data_ptr(), ws.data_ptr(),
                                           ws.numel() * 4, _native.stream_ptr(dev)), "drt_score_ce_fwd")
        ctx.save_for_backward(qf, pf, S, lse)
        ctx.target_stride = int(target_stride)
        ctx.scale = float(scale)
        ctx.in_dtypes = (q.dtype, p.dtype)
        ctx.mark_non_differentiable(S)
        return loss, S

    @staticmethod
    def backward(ctx, g_loss, g_scores):
        qf, pf, S, lse = ctx.saved_tensors
        lib = _native.load()
        m, n = S.shape
        d = qf.shape[1]
        dev = S.device
        g = g_loss.detach().to(torch.float32).contiguous().reshape(1)
        dq = torch.empty((m, d), dtype=torch.float32, device=dev)
        dp = torch.empty((n, d), dtype=torch.float32, device=dev)
        ws = _workspace(lib, m, n, d, dev)
        _native.check(lib.drt_score_ce_bwd(qf.data_ptr(), pf.data_ptr(), S.data_ptr(), lse.data_ptr(), m, n, d,
                                           ctx.target_stride, g.data_ptr(), ctx.scale, dq.data_ptr(), dp.data_ptr(),
                                           ws.data_ptr(), ws.numel() * 4, _native.stream_ptr(dev)),
                      "drt_score_ce_bwd")
        if ctx.in_dtypes[0] != torch.float32:
            dq = dq.to(ctx.in_dtypes[0])
        if ctx.in_dtypes[1] != torch.float32:
            dp = dp.to(ctx.in_dtypes[1])
        return dq, dp, None, None


def score_ce(q: torch.Tensor, p: torch.Tensor, target_stride: int, scale: float = 1.0):
    """(loss, scores) for in-batch negatives with target_i = i * target_stride."""
    return ScoreCE.apply(q, p, target_stride, scale)
