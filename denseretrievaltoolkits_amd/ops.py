"""``torch.ops.drt.*``: the PyTorch-ROCm custom operators of the hot path.

The operators are defined in C++ (csrc/torch_ops.cpp, ``TORCH_LIBRARY(drt, ...)``, built into
``_drt_ops.so`` next to ``libdrt_hip.so``) over the C ABI of ``include/drt.h``.  This module
loads that library (no fallback: a missing library raises) and registers, per operator, the
fake (meta) implementation that torch.compile / FakeTensor tracing need, plus the autograd
formula of the fused score + cross-entropy op.

    torch.ops.drt.ip_topk(q, p, k, id_offset, stats)   -> (scores, ids, status)   index.py:31-33
    torch.ops.drt.ip_topk_resolve(q, p, k, off, s, i, st, stats) -> n_resolved  (in place, synchronous)
    torch.ops.drt.row_stats / refine_delta / refine_sort  (canonical exact-score order, include/drt.h)
    torch.ops.drt.topk_merge(scores, ids, k_out)        -> (scores, ids)           utils.py:215-229
    torch.ops.drt.ip_topk_large(_keys) / merge_exact    (k > 2048; sharded: merged by exact order keys)
    torch.ops.drt.dist_sample / dist_tau / dist_filter / dist_filter_chunks_into / dist_filter_lists / merge_packed
                                                                                            (sharded, §8e)
    torch.ops.drt.score_ce_fwd(q, p, stride, scale)     -> (loss, scores, lse)     biencoder.py:107-119
    torch.ops.drt.score_ce_bwd(g, q, p, scores, lse, stride, scale) -> (dq, dp)
    torch.ops.drt.embed_ln / linear / attention / layernorm / pool / l2_normalize  (BertModel pieces)
"""
from __future__ import annotations

import os
import threading

import torch

from . import _native
from ._native import ROW_STATS_LEN
from .build_native import OPS_LIB_PATH

_lock = threading.Lock()
_loaded = False


def load():
    """Load the custom-op library once (after libdrt_hip.so, whose copy it then shares)."""
    global _loaded
    if _loaded:
        return torch.ops.drt
    with _lock:
        if _loaded:
            return torch.ops.drt
        _native.load()
        if not os.path.exists(OPS_LIB_PATH):
            raise RuntimeError(f"torch custom-op library not found at {OPS_LIB_PATH}; build it with "
                               "`python -m denseretrievaltoolkits_amd.build_native` (no CPU fallback exists)")
        torch.ops.load_library(OPS_LIB_PATH)
        _register_python_parts()
        _loaded = True
    return torch.ops.drt


def _register_python_parts():
    lib = torch.library

    @lib.register_fake("drt::ip_topk")
    def _(q, p, k, id_offset=0, stats=None):
        nq = q.shape[0]
        return (q.new_empty((nq, k), dtype=torch.float32), q.new_empty((nq, k), dtype=torch.int64),
                q.new_empty((nq,), dtype=torch.int32))

    @lib.register_fake("drt::ip_topk.out")
    def _(q, p, k, id_offset, stats=None, *, scores, ids, status):
        return None

    @lib.register_fake("drt::ip_topk_resolve")
    def _(q, p, k, id_offset, scores, ids, status, stats=None):
        # the count of rescanned queries is data-dependent (it reads the status back)
        return torch.library.get_ctx().new_dynamic_size()

    @lib.register_fake("drt::ip_topk_resolve_wide")
    def _(q, p, k, id_offset, scores, ids, status, stats):
        return torch.library.get_ctx().new_dynamic_size()

    @lib.register_fake("drt::ip_topk_large")
    def _(q, p, k, id_offset, stats, tau):
        nq = q.shape[0]
        return (q.new_empty((nq, k), dtype=torch.float32), q.new_empty((nq, k), dtype=torch.int64),
                q.new_empty((nq,), dtype=torch.int32))

    @lib.register_fake("drt::ip_topk_large_keys")
    def _(q, p, k, id_offset, stats, tau):
        nq = q.shape[0]
        return (q.new_empty((nq, k), dtype=torch.float32), q.new_empty((nq, k), dtype=torch.int64),
                q.new_empty((nq,), dtype=torch.int32), q.new_empty((nq, k), dtype=torch.int64))

    @lib.register_fake("drt::merge_exact")
    def _(keys, ids, k):
        nq = keys.shape[1]
        return keys.new_empty((nq, k), dtype=torch.float32), ids.new_empty((nq, k))

    @lib.register_fake("drt::row_stats")
    def _(p, prev=None):
        return p.new_empty((ROW_STATS_LEN,), dtype=torch.float32)

    @lib.register_fake("drt::refine_delta")
    def _(q, p, row_offset, cand_scores, cand_ids, k, stats, tau, status, local=False):
        return cand_scores.new_empty(cand_scores.shape), cand_scores.new_empty((cand_scores.shape[0], 2),
                                                                                 dtype=torch.int32)

    @lib.register_fake("drt::refine_sort")
    def _(cand_scores, cand_ids, delta, cnt, k):
        nq = cand_scores.shape[0]
        return cand_scores.new_empty((nq, k)), cand_ids.new_empty((nq, k))

    @lib.register_fake("drt::topk_merge")
    def _(scores, ids, k_out):
        nq = scores.shape[1]
        return scores.new_empty((nq, k_out)), ids.new_empty((nq, k_out))

    @lib.register_fake("drt::dist_sample")
    def _(q, p, n_global, k):
        r = int(_native.load().drt_ip_topk_sample_rank(k))
        return q.new_empty((q.shape[0], r), dtype=torch.int32)

    @lib.register_fake("drt::dist_tau")
    def _(lists, k):
        return lists.new_empty((lists.shape[1],), dtype=torch.float32)

    @lib.register_fake("drt::dist_filter")
    def _(q, p, n_global, k, id_offset, tau):
        return q.new_empty((q.shape[0], k + 1), dtype=torch.int64)

    @lib.register_fake("drt::dist_filter_lists")
    def _(q, p, n_global, k, id_offset, lists):
        return q.new_empty((q.shape[0], k + 1), dtype=torch.int64)

    @lib.register_fake("drt::dist_filter_into")
    def _(q, p, n_global, k, id_offset, tau, packed):
        return None

    @lib.register_fake("drt::dist_filter_chunks_into")
    def _(q, p, n_global, k, id_offset, tau, starts, packed):
        return None

    @lib.register_fake("drt::dist_filter_lists_into")
    def _(q, p, n_global, k, id_offset, lists, q0, packed):
        return None

    @lib.register_fake("drt::merge_packed")
    def _(parts, k, n_global, k_cert=-1):
        nq = parts.shape[1]
        return (parts.new_empty((nq, k), dtype=torch.float32), parts.new_empty((nq, k), dtype=torch.int64),
                parts.new_empty((nq,), dtype=torch.int32))

    @lib.register_fake("drt::score_ce_fwd")
    def _(q, p, target_stride, scale):
        return q.new_empty(()), q.new_empty((q.shape[0], p.shape[0])), q.new_empty((q.shape[0],))

    @lib.register_fake("drt::score_ce_bwd")
    def _(grad, q, p, scores, lse, target_stride, scale):
        return q.new_empty(q.shape), p.new_empty(p.shape)

    @lib.register_fake("drt::embed_ln")
    def _(input_ids, token_type_ids, word, pos, type, gamma, beta, eps):
        return input_ids.new_empty(tuple(input_ids.shape) + (word.shape[1],), dtype=torch.bfloat16)

    @lib.register_fake("drt::linear")
    def _(x, w, bias, residual, gelu=False, fp32_out=False):
        return x.new_empty((x.shape[0], w.shape[0]), dtype=torch.float32 if fp32_out else torch.bfloat16)

    @lib.register_fake("drt::attention")
    def _(qkv, mask, batch, heads, scale):
        return qkv.new_empty((qkv.shape[0], qkv.shape[1] // 3))

    @lib.register_fake("drt::layernorm")
    def _(x, gamma, beta, eps):
        return x.new_empty(x.shape, dtype=torch.bfloat16)

    @lib.register_fake("drt::pool")
    def _(hidden, mask, mode):
        return hidden.new_empty((hidden.shape[0], hidden.shape[2]), dtype=torch.float32)

    @lib.register_fake("drt::l2_normalize")
    def _(x):
        return x.new_empty(x.shape)

    # autograd of the fused score + CE: only the loss is differentiable (scores / lse are
    # returned for the caller and for the backward, like DRModel.forward's `scores`)
    def setup_context(ctx, inputs, output):
        q, p, target_stride, scale = inputs
        _, scores, lse = output
        ctx.save_for_backward(q, p, scores, lse)
        ctx.target_stride = int(target_stride)
        ctx.scale = float(scale)
        ctx.mark_non_differentiable(scores, lse)

    def backward(ctx, g_loss, g_scores, g_lse):
        q, p, scores, lse = ctx.saved_tensors
        dq, dp = torch.ops.drt.score_ce_bwd(g_loss, q, p, scores, lse, ctx.target_stride, ctx.scale)
        return dq, dp, None, None

    lib.register_autograd("drt::score_ce_fwd", backward, setup_context=setup_context)
