"""ctypes binding of the C-ABI in ``include/drt.h`` (``libdrt_hip.so``).

The product path has no CPU fallback: if the library is missing or cannot be
loaded, every op raises.  ``torch`` is imported first so that the HIP runtime
the library links against (SONAME libamdhip64.so.7) resolves to the one torch
already loaded — one runtime, one set of streams.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

from .build_native import LIB_PATH

DRT_OK = 0
DRT_EINVAL = -1
ROW_STATS_LEN = 34   # DRT_ROW_STATS_LEN (include/drt.h): floats of drt_row_stats_bf16's statistics

_lock = threading.Lock()
_lib = None

c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_sz = ctypes.c_size_t
c_vp = ctypes.c_void_p
c_f32 = ctypes.c_float
c_u64 = ctypes.c_uint64

# (name, restype, argtypes) — one line per entry point of include/drt.h
_SIGNATURES = [
    ("drt_version", ctypes.c_char_p, []),
    ("drt_ip_topk_workspace", c_sz, [c_i64, c_i64, c_i32, c_i32]),
    ("drt_ip_topk_bf16", c_i32, [c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    ("drt_ip_topk_resolve_workspace", c_sz, [c_i64, c_i64, c_i32]),
    ("drt_ip_topk_resolve", c_i32, [c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_sz,
                                    c_vp, c_vp]),
    ("drt_topk_merge", c_i32, [c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp]),
    ("drt_ip_topk_sample_rank", c_i32, [c_i32]),
    ("drt_ip_topk_dist_workspace", c_sz, [c_i64, c_i64, c_i64, c_i32, c_i32]),
    ("drt_ip_topk_dist_sample", c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_sz, c_vp]),
    ("drt_ip_topk_dist_tau", c_i32, [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp]),
    ("drt_ip_topk_dist_filter", c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp,
                                        c_sz, c_vp]),
    ("drt_ip_topk_dist_filter_chunks", c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i32, c_i64, c_vp, c_vp,
                                               c_vp, c_i32, c_vp, c_sz, c_vp]),
    ("drt_ip_topk_dist_filter_lists", c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i32, c_i64, c_vp, c_i32,
                                              c_vp, c_vp, c_vp, c_sz, c_vp]),
    ("drt_ip_topk_dist_filter_lists_at", c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i32, c_i64, c_vp,
                                                 c_i32, c_i64, c_vp, c_vp, c_vp, c_sz, c_vp]),
    ("drt_topk_merge_packed", c_i32, [c_vp, c_i64, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp]),
    ("drt_topk_merge_packed_cert", c_i32, [c_vp, c_i64, c_i32, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp]),
    ("drt_topk_merge_packed_capped", c_i32, [c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp,
                                             c_vp]),
    ("drt_row_stats_bf16", c_i32, [c_vp, c_i64, c_i32, c_vp, c_i32, c_vp]),
    ("drt_refine_width", c_i32, [c_i32]),
    ("drt_ip_topk_exact_bf16", c_i32, [c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                       c_sz, c_vp]),
    ("drt_hit_metrics_i8", c_i32, [c_vp, c_i64, c_i64, c_vp, c_i32, c_vp, c_vp]),
    ("drt_answer_match_i32", c_i32, [c_vp, c_i32, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i32, c_i32, c_vp,
                                     c_vp, c_vp]),
    ("drt_ip_topk_resolve_exact", c_i32, [c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp,
                                          c_vp, c_sz, c_vp, c_vp]),
    ("drt_ip_topk_resolve_wide_workspace", c_sz, [c_i64, c_i32]),
    ("drt_ip_topk_resolve_wide", c_i32, [c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp,
                                         c_vp, c_sz, c_vp, c_vp]),
    ("drt_ip_topk_large_workspace", c_sz, [c_i32, c_i32]),
    ("drt_ip_topk_large", c_i32, [c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                  c_sz, c_vp]),
    ("drt_ip_topk_large_keys", c_i32, [c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                       c_vp, c_vp, c_sz, c_vp]),
    ("drt_merge_exact", c_i32, [c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp]),
    ("drt_refine_delta_bf16", c_i32, [c_vp, c_i64, c_i32, c_vp, c_i64, c_i64, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp,
                                      c_vp, c_vp, c_vp, c_vp]),
    ("drt_refine_delta_local_bf16", c_i32, [c_vp, c_i64, c_i32, c_vp, c_i64, c_i64, c_vp, c_vp, c_i32, c_i32, c_vp,
                                            c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("drt_refine_sort", c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp]),
    ("drt_gemm_nt_bf16_f32", c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i64, c_vp]),
    ("drt_embed_ln", c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_i32, c_vp, c_vp]),
    ("drt_linear_bf16", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i32, c_vp]),
    ("drt_linear_workspace", c_sz, [c_i64, c_i64, c_i64]),
    ("drt_linear_bf16_ws", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i32, c_vp, c_sz, c_vp]),
    ("drt_linear_ln_bf16_ws", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp, c_vp, c_i64, c_i64, c_i64,
                                      c_vp, c_sz, c_vp]),
    ("drt_layernorm_f32_bf16", c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_f32, c_vp, c_vp]),
    ("drt_attention_fwd_lse_bf16", c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i32, c_f32, c_vp]),
    ("drt_layernorm_bwd_workspace", c_sz, [c_i64, c_i32]),
    ("drt_layernorm_bwd_drop_bf16", c_i32, [c_vp, c_vp, c_vp, c_f32, c_i64, c_i32, c_vp, c_vp, c_vp, c_f32, c_u64,
                                            c_u64, c_vp, c_vp, c_vp, c_sz, c_vp]),
    ("drt_layernorm_bwd_sum_bf16", c_i32, [c_vp, c_vp, c_vp, c_f32, c_i64, c_i32, c_vp, c_vp, c_vp, c_f32, c_u64,
                                           c_u64, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    ("drt_linear_bf16_ex", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i32, c_f32, c_u64,
                                   c_u64, c_vp, c_sz, c_vp]),
    ("drt_layernorm_bwd_bf16", c_i32, [c_vp, c_vp, c_vp, c_f32, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz,
                                       c_vp]),
    ("drt_colsum_workspace", c_sz, [c_i64, c_i64]),
    ("drt_colsum_bf16", c_i32, [c_vp, c_i64, c_i64, c_vp, c_vp, c_sz, c_vp]),
    ("drt_colsum_f32", c_i32, [c_vp, c_i64, c_i64, c_vp, c_vp, c_sz, c_vp]),
    ("drt_linear_dgelu_bias_workspace", c_sz, [c_i64, c_i64, c_i64]),
    ("drt_linear_dgelu_bias_bf16", c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_sz, c_vp]),
    ("drt_gelu_bwd_bf16", c_i32, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    ("drt_linear_wgrad_workspace", c_sz, [c_i64, c_i64, c_i64]),
    ("drt_linear_wgrad_bf16", c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_sz, c_vp]),
    ("drt_transpose_bf16", c_i32, [c_vp, c_i64, c_i64, c_vp, c_vp]),
    ("drt_transpose_bf16_ld", c_i32, [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp]),
    ("drt_embed_ln_pre", c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_i32, c_vp, c_vp,
                                 c_vp]),
    ("drt_gelu_bf16", c_i32, [c_vp, c_i64, c_vp, c_vp]),
    ("drt_embedding_bwd", c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp]),
    ("drt_embedding_bwd_types", c_i32, [c_vp, c_vp, c_i32, c_vp, c_i64, c_i64, c_i32, c_i64, c_vp, c_vp, c_vp,
                                         c_vp]),
    ("drt_attention_train_fwd_bf16", c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i32, c_f32, c_f32,
                                             ctypes.c_uint64, ctypes.c_uint64, c_vp]),
    ("drt_attention_train_bwd_bf16", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i32, c_f32,
                                             c_f32, ctypes.c_uint64, ctypes.c_uint64, c_vp]),
    ("drt_dropout_add_bf16", c_i32, [c_vp, c_vp, c_i64, c_f32, ctypes.c_uint64, ctypes.c_uint64, c_vp, c_vp]),
    ("drt_attention_train_fwd_bits_bf16", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i32, c_f32,
                                                  c_f32, c_u64, c_u64, c_vp]),
    ("drt_attention_train_bwd_bits_bf16", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32,
                                                  c_i32, c_f32, c_f32, c_u64, c_u64, c_vp]),
    ("drt_attention_train_bwd_bias_workspace", c_sz, [c_i64, c_i32, c_i32]),
    ("drt_attention_train_bwd_bias_bf16", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32,
                                                  c_i32, c_f32, c_f32, c_u64, c_u64, c_vp, c_vp, c_sz, c_vp]),
    ("drt_attention_bwd_bf16", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i32, c_f32, c_vp]),
    ("drt_layernorm_bf16", c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_f32, c_vp, c_vp]),
    ("drt_attention_bf16", c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i32, c_f32, c_vp]),
    ("drt_pool_bf16", c_i32, [c_vp, c_vp, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp]),
    ("drt_l2_normalize_f32", c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp]),
    ("drt_gemm_nt_f32", c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp]),
    ("drt_gemm_f32", c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp]),
    ("drt_ce_fwd", c_i32, [c_vp, c_i64, c_i64, c_i64, c_f32, c_vp, c_vp, c_vp, c_vp]),
    ("drt_ce_bwd", c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_f32, c_vp, c_vp]),
    ("drt_score_ce_workspace", c_sz, [c_i64, c_i64, c_i32]),
    ("drt_score_ce_fwd", c_i32, [c_vp, c_vp, c_i64, c_i64, c_i32, c_i64, c_f32, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    ("drt_score_ce_bwd", c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i64, c_vp, c_f32, c_vp, c_vp, c_vp,
                                 c_sz, c_vp]),
    ("drt_transpose_f32", c_i32, [c_vp, c_i64, c_i64, c_vp, c_vp]),
    ("drt_profile_enable", c_i32, [c_i32, c_i32]),
    ("drt_profile_read", c_i32, [c_i32, c_vp, c_vp]),
    ("drt_profile_read_each", c_i32, [c_i32, c_vp, c_i64, c_vp]),
]

PROF_SCAN, PROF_SAMPLE, PROF_SELECT, PROF_MERGE, PROF_GEMM = range(5)

EXPORTED = [n for n, _, _ in _SIGNATURES]


def lib_path() -> str:
    return os.environ.get("DRT_LIB", LIB_PATH)


def load():
    """Load (once) and return the ctypes handle. Raises if the library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = lib_path()
        if not os.path.exists(path):
            raise RuntimeError(
                f"DRT native library not found at {path}; build it with "
                "`python -m denseretrievaltoolkits_amd.build_native` (no CPU fallback exists)")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        for name, res, args in _SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc: int, what: str) -> None:
    if rc != DRT_OK:
        if rc == DRT_EINVAL:
            raise ValueError(f"{what}: invalid argument (DRT_EINVAL)")
        raise RuntimeError(f"{what}: HIP error {rc}")


def stream_ptr(device=None) -> int:
    """hipStream_t of torch's current stream on `device` (the stream ops enqueue on)."""
    return torch.cuda.current_stream(device).cuda_stream
