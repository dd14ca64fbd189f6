"""Backward building blocks of the HIP encoder tower, used by the
training tower (model/train_tower.py).

The training step of run_random_sampling.py (DRT/trainer/trainer.py:113-133) differentiates
HF ``BertModel`` under autograd; these functions restate the gradients of its ops on the HIP
kernels for the bf16 activations the HIP forward stores:

* ``linear_backward``   nn.Linear: dX = dY W (the NT GEMM against a transposed weight copy),
                        dW = dY^T X (``wgrad``: the TN GEMM reading both token-major operands
                        directly, deterministic split over tokens, fp32 output), db = column
                        sums of dY;
* ``layernorm_backward`` / ``gelu_backward``: thin wrappers of the C-ABI entries
                        (include/drt.h).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .. import _native


def _ws(nbytes: int, dev) -> Optional[torch.Tensor]:
    return torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=dev) if nbytes else None


def _ptr(t: Optional[torch.Tensor]):
    return t.data_ptr() if t is not None else None


def transpose_bf16(x: torch.Tensor, cols_pad: int = 0) -> torch.Tensor:
    """x [R, C] bf16 -> x^T [C, R + pad] with zero padding columns (k-contiguous GEMM operand)."""
    lib = _native.load()
    R, C = x.shape
    y = torch.empty((C, R + cols_pad), dtype=torch.bfloat16, device=x.device)
    if cols_pad:
        y[:, R:].zero_()
    _native.check(lib.drt_transpose_bf16_ld(x.data_ptr(), R, C, y.data_ptr(), R + cols_pad,
                                            _native.stream_ptr(x.device)), "drt_transpose_bf16_ld")
    return y


def colsum(x: torch.Tensor) -> torch.Tensor:
    lib = _native.load()
    M, N = x.shape
    out = torch.empty(N, dtype=torch.float32, device=x.device)
    nb = int(lib.drt_colsum_workspace(M, N))
    ws = _ws(nb, x.device)
    _native.check(lib.drt_colsum_bf16(x.data_ptr(), M, N, out.data_ptr(), _ptr(ws), nb,
                                      _native.stream_ptr(x.device)), "drt_colsum_bf16")
    return out


def linear_backward(dy: torch.Tensor, x: torch.Tensor, w_t: torch.Tensor, want_dx: bool = True,
                    resid: Optional[torch.Tensor] = None, gelu_pre: Optional[torch.Tensor] = None,
                    db: Optional[torch.Tensor] = None, dx_colsum: Optional[torch.Tensor] = None
                    ) -> Tuple[Optional[torch.Tensor], torch.Tensor, torch.Tensor]:
    """Gradients of y = x W^T + b (nn.Linear, W [N, K]) for dy [T, N], x [T, K] (bf16 CUDA),
    given w_t = W^T [K, N] bf16.  Returns (dx bf16 [T, K] or None, dW fp32 [N, K], db fp32 [N]);
    ``resid`` [T, K] bf16 is added to dx in the dgrad GEMM's epilogue (a residual branch);
    ``gelu_pre`` [T, K] (x = GELU(gelu_pre)) makes dx the gradient of gelu_pre instead, the GELU
    backward applied in the same epilogue (drt_linear_bf16_ex); ``db``: the bias gradient already
    produced by dy's producer (the LayerNorm / attention backward), returned as is instead of a
    column-sum pass over dy.  ``dx_colsum`` [K] fp32 (with ``gelu_pre``): also filled with the column
    sums of dx -- the bias gradient of the GELU's linear -- from the dgrad GEMM's epilogue
    (drt_linear_dgelu_bias_bf16)."""
    lib = _native.load()
    dev = dy.device
    s = _native.stream_ptr(dev)
    T, N = dy.shape
    K = x.shape[1]
    if N % 64 or K % 64:
        raise ValueError("linear_backward: feature sizes must be multiples of 64")
    dx = None
    if want_dx:
        dx = torch.empty((T, K), dtype=torch.bfloat16, device=dev)
        nb = int(lib.drt_linear_workspace(T, K, N))
        ws = _ws(nb, dev)
        if gelu_pre is not None and dx_colsum is not None:
            if resid is not None:
                raise ValueError("linear_backward: gelu_pre and resid are exclusive")
            nb = int(lib.drt_linear_dgelu_bias_workspace(T, K, N))
            ws = _ws(nb, dev)
            _native.check(lib.drt_linear_dgelu_bias_bf16(dy.data_ptr(), w_t.data_ptr(), gelu_pre.data_ptr(),
                                                         dx.data_ptr(), T, K, N, dx_colsum.data_ptr(), _ptr(ws), nb,
                                                         s), "dgrad (GELU backward + bias gradient epilogue)")
        elif gelu_pre is not None:
            if resid is not None:
                raise ValueError("linear_backward: gelu_pre and resid are exclusive")
            _native.check(lib.drt_linear_bf16_ex(dy.data_ptr(), w_t.data_ptr(), None, None, gelu_pre.data_ptr(),
                                                 dx.data_ptr(), None, T, K, N, 0, 0.0, 0, 0, _ptr(ws), nb, s),
                          "dgrad (GELU backward epilogue)")
        else:
            _native.check(lib.drt_linear_bf16_ws(dy.data_ptr(), w_t.data_ptr(), None, _ptr(resid), dx.data_ptr(), T, K,
                                                 N, 0, _ptr(ws), nb, s), "dgrad")
    dW = wgrad(dy, x)
    return dx, dW, (db if db is not None else colsum(dy))


WGRAD_TN = True   # A/B switch: False = transposed operand copies + NT GEMM (the round-1 path)


def wgrad(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dW [N, K] fp32 = dy[T, N]^T x[T, K].  Token counts that are multiples of 32 go straight to
    the TN GEMM (drt_linear_wgrad_bf16, no transposed copies); others transpose both operands
    (zero-padded to 64 tokens) and run the NT GEMM."""
    lib = _native.load()
    dev = dy.device
    s = _native.stream_ptr(dev)
    T, N = dy.shape
    K = x.shape[1]
    dW = torch.empty((N, K), dtype=torch.float32, device=dev)
    if WGRAD_TN and T % 32 == 0:
        nb = int(lib.drt_linear_wgrad_workspace(T, N, K))
        ws = _ws(nb, dev)
        _native.check(lib.drt_linear_wgrad_bf16(dy.data_ptr(), x.data_ptr(), dW.data_ptr(), T, N, K, _ptr(ws), nb, s),
                      "drt_linear_wgrad_bf16")
        return dW
    pad = (-T) % 64
    dyT = transpose_bf16(dy, pad)        # [N, T64]
    xT = transpose_bf16(x, pad)          # [K, T64]
    T64 = T + pad
    nb = int(lib.drt_linear_workspace(N, K, T64))
    ws = _ws(nb, dev)
    _native.check(lib.drt_linear_bf16_ws(dyT.data_ptr(), xT.data_ptr(), None, None, dW.data_ptr(), N, K, T64, 2,
                                         _ptr(ws), nb, s), "wgrad")
    return dW


def layernorm_backward(dy: torch.Tensor, x: torch.Tensor, gamma: torch.Tensor, eps: float,
                       dres: Optional[torch.Tensor] = None, drop=None, want_sum: bool = False):
    """(dx bf16 [M, H], dgamma fp32 [H], dbeta fp32 [H]) of out = LN(x) (x = the bf16 pre-LN sums).
    ``drop`` = (p, seed, site): also return dropout(dx) with that mask (drt_layernorm_bwd_drop_bf16)
    as a fourth value.  ``want_sum``: also return (last) the column sums of the gradient handed
    down -- dropout(dx), or dx -- i.e. the bias gradient of the linear below
    (drt_layernorm_bwd_sum_bf16)."""
    lib = _native.load()
    M, H = x.shape
    dev = x.device
    dx = torch.empty((M, H), dtype=torch.bfloat16, device=dev)
    dg = torch.empty(H, dtype=torch.float32, device=dev)
    db = torch.empty(H, dtype=torch.float32, device=dev)
    nb = int(lib.drt_layernorm_bwd_workspace(M, H))
    ws = _ws(nb, dev)
    dxd = torch.empty_like(dx) if drop is not None else None
    p, seed, site = drop if drop is not None else (0.0, 0, 0)
    dsum = torch.empty(H, dtype=torch.float32, device=dev) if want_sum else None
    _native.check(lib.drt_layernorm_bwd_sum_bf16(dy.data_ptr(), x.data_ptr(), gamma.data_ptr(), float(eps), M, H,
                                                 _ptr(dres), dx.data_ptr(), _ptr(dxd), float(p), seed, site,
                                                 dg.data_ptr(), db.data_ptr(), _ptr(dsum), _ptr(ws), nb,
                                                 _native.stream_ptr(dev)), "drt_layernorm_bwd_sum_bf16")
    out = (dx, dg, db) + ((dxd,) if drop is not None else ()) + ((dsum,) if want_sum else ())
    return out


def gelu_backward(dy: torch.Tensor, pre: torch.Tensor) -> torch.Tensor:
    lib = _native.load()
    dx = torch.empty_like(dy)
    _native.check(lib.drt_gelu_bwd_bf16(dy.data_ptr(), pre.data_ptr(), dy.numel(), dx.data_ptr(),
                                        _native.stream_ptr(dy.device)), "drt_gelu_bwd_bf16")
    return dx
