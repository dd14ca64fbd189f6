"""Training forward + backward of a BERT tower on the HIP kernels.

The reference differentiates HF ``BertModel`` under autograd in every training step
(DRT/trainer/trainer.py:113-133 -> DRModel.forward, DRT/model/biencoder.py:88-125).  Here one
``torch.autograd.Function`` per BertLayer (plus one for the embeddings) runs the tower, so each
layer's parameter gradients reach autograd -- and DDP's bucketed all-reduce -- as soon as that
layer's backward is done: the forward on the inference kernels plus the activations the backward needs (bf16: layer input, qkv, ctx, attention LSE, pre-LN sums,
post-LN1, FFN pre-/post-activation), and the backward entirely on HIP kernels:

    LN2 bwd -> FFN2 linear bwd -> GELU bwd -> FFN1 linear bwd (+ dx2 residual in the dgrad
    epilogue) -> LN1 bwd -> O-proj linear bwd -> attention bwd -> QKV linear bwd (+ dx1)
    ... -> embedding LN bwd -> word / position / type scatter-add

producing fp32 gradients for every HF parameter (QKV split back into query/key/value).
Dropout as HF applies it in train mode (embeddings output, attention probabilities, both
sublayer outputs before their residual add; hidden_dropout_prob / attention_probs_dropout_prob):
each keep is a counter-based hash of (per-call seed, site, element index) (csrc/drt_common.h
drop_hash24; the attention probabilities draw two keeps per 32-bit hash of (row key, key pair),
attn_row_key / attn_mix), so the backward regenerates the hidden-site masks instead of storing them
and reads the attention keep bits the forward wrote (1 bit per probability); the seed comes from torch's CPU generator (``torch.manual_seed`` makes a step reproducible).  The
masks are not HF's Philox stream: same distribution and semantics, different draws.
Scope: L <= 512 (BERT max_position_embeddings; L <= 160 -- the recipe, p_max_len 156 -- runs the whole-sequence
attention backward, longer sequences the streamed one), erf GELU, head_dim 64; anything else
raises.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

from .. import _native
from .encoder import BertShape, _check_supported
from .encoder_bwd import _ptr, layernorm_backward, linear_backward

MAX_TRAIN_SEQ = 512


def tower_supported(model) -> Optional[str]:
    """None if the HIP training tower can run this HF BertModel, else the reason."""
    cfg = model.config
    if type(model).__name__ != "BertModel":
        return f"{type(model).__name__} is not a BertModel"
    try:
        _check_supported(BertShape.from_config(cfg))
    except ValueError as e:
        return str(e)
    return None


class _Weights:
    """bf16 copies (and transposes) of the tower's linears for one step; fp32 LN / bias / tables."""

    def __init__(self, model, dev):
        lib = _native.load()
        sd = dict(model.named_parameters())
        self.names = list(sd.keys())
        self.sd = sd
        self.layers = []
        s = _native.stream_ptr(dev)

        def b16(t):
            return t.detach().to(torch.bfloat16).contiguous()

        def tr(w):   # [N, K] bf16 -> [K, N]
            n, k = w.shape
            y = torch.empty((k, n), dtype=torch.bfloat16, device=dev)
            _native.check(lib.drt_transpose_bf16(w.data_ptr(), n, k, y.data_ptr(), s), "drt_transpose_bf16")
            return y

        nl = model.config.num_hidden_layers
        for i in range(nl):
            p = f"encoder.layer.{i}."
            wqkv = b16(torch.cat([sd[p + f"attention.self.{n}.weight"].detach() for n in ("query", "key", "value")]))
            bqkv = torch.cat([sd[p + f"attention.self.{n}.bias"].detach() for n in ("query", "key", "value")]).float()
            wo = b16(sd[p + "attention.output.dense.weight"])
            wi = b16(sd[p + "intermediate.dense.weight"])
            wf = b16(sd[p + "output.dense.weight"])
            self.layers.append(dict(
                wqkv=wqkv, wqkv_t=tr(wqkv), bqkv=bqkv.contiguous(),
                wo=wo, wo_t=tr(wo), bo=sd[p + "attention.output.dense.bias"].detach().float().contiguous(),
                g1=sd[p + "attention.output.LayerNorm.weight"].detach().float().contiguous(),
                b1=sd[p + "attention.output.LayerNorm.bias"].detach().float().contiguous(),
                wi=wi, wi_t=tr(wi), bi=sd[p + "intermediate.dense.bias"].detach().float().contiguous(),
                wf=wf, wf_t=tr(wf), bf=sd[p + "output.dense.bias"].detach().float().contiguous(),
                g2=sd[p + "output.LayerNorm.weight"].detach().float().contiguous(),
                b2=sd[p + "output.LayerNorm.bias"].detach().float().contiguous(),
            ))
        e = "embeddings."
        self.word = sd[e + "word_embeddings.weight"].detach().float().contiguous()
        self.pos = sd[e + "position_embeddings.weight"].detach().float().contiguous()
        self.type = sd[e + "token_type_embeddings.weight"].detach().float().contiguous()
        self.emb_g = sd[e + "LayerNorm.weight"].detach().float().contiguous()
        self.emb_b = sd[e + "LayerNorm.bias"].detach().float().contiguous()


def _lin(lib, x, w, b, out, resid=None, gelu=False, stream=None, pre_out=None, drop=None):
    """out = x W^T + b (GELU) (+ resid); ``pre_out``: also store the pre-activation (GELU);
    ``drop`` = (p, seed, site): out = dropout(x W^T + b) + resid (drt_linear_bf16_ex epilogues)."""
    m, k = x.shape
    n = w.shape[0]
    flags = (1 if gelu else 0) | (2 if out.dtype == torch.float32 else 0)
    nb = int(lib.drt_linear_workspace(m, n, k))
    ws = torch.empty((nb + 3) // 4, dtype=torch.float32, device=x.device) if nb else None
    if pre_out is not None or drop is not None:
        p, seed, site = drop if drop is not None else (0.0, 0, 0)
        _native.check(lib.drt_linear_bf16_ex(x.data_ptr(), w.data_ptr(), _ptr(b), _ptr(resid), None, out.data_ptr(),
                                             _ptr(pre_out), m, n, k, flags | (4 if drop is not None else 0), float(p),
                                             seed, site, _ptr(ws), nb, stream), "drt_linear_bf16_ex")
        return out
    _native.check(lib.drt_linear_bf16_ws(x.data_ptr(), w.data_ptr(), _ptr(b), _ptr(resid), out.data_ptr(), m, n, k,
                                         flags, _ptr(ws), nb, stream), "drt_linear_bf16_ws")
    return out


def _layernorm(lib, x, g, b, eps, stream):
    out = torch.empty_like(x)
    _native.check(lib.drt_layernorm_bf16(x.data_ptr(), x.shape[0], x.shape[1], g.data_ptr(), b.data_ptr(), eps,
                                         out.data_ptr(), stream), "drt_layernorm_bf16")
    return out


def _dropout(lib, y, p, seed, site, stream, resid=None):
    out = torch.empty_like(y)
    _native.check(lib.drt_dropout_add_bf16(y.data_ptr(), _ptr(resid), y.numel(), float(p), seed, site,
                                           out.data_ptr(), stream), "drt_dropout_add_bf16")
    return out


def dropout_sites(layer: int):
    """(attention probabilities, attention output, FFN output) site ids of a layer; 0 = embeddings."""
    return 4 * layer + 1, 4 * layer + 2, 4 * layer + 3


class _Step:
    """What every node of one tower pass shares: weights, shape, masks' inputs, dropout."""

    def __init__(self, model, W: _Weights, ids, mask, drop, types=None):
        cfg = model.config
        self.model, self.W, self.ids, self.mask, self.drop = model, W, ids, mask, drop
        self.types = types   # token_type_ids [B, L] int64 or None (all type 0)
        self.B, self.L = ids.shape
        self.H, self.heads, self.eps = cfg.hidden_size, cfg.num_attention_heads, float(cfg.layer_norm_eps)
        self.scale = 1.0 / (self.H // self.heads) ** 0.5
        self.dev = ids.device


def embed_forward(st: _Step):
    """h0 = dropout(LN(word + pos + type)) bf16 [T, H] and the pre-LN sum the backward needs."""
    lib = _native.load()
    s = _native.stream_ptr(st.dev)
    W = st.W
    T = st.B * st.L
    h = torch.empty((T, st.H), dtype=torch.bfloat16, device=st.dev)
    emb_pre = torch.empty_like(h)
    _native.check(lib.drt_embed_ln_pre(st.ids.data_ptr(), _ptr(st.types), st.B, st.L, W.word.data_ptr(),
                                       W.pos.data_ptr(),
                                       W.type.data_ptr(), W.emb_g.data_ptr(), W.emb_b.data_ptr(), st.eps, st.H,
                                       h.data_ptr(), emb_pre.data_ptr(), s), "drt_embed_ln_pre")
    ph, _, seed = st.drop
    if ph > 0:
        h = _dropout(lib, h, ph, seed, 0, s)
    return h, emb_pre


def embed_backward(st: _Step, emb_pre, d) -> Dict[str, torch.Tensor]:
    lib = _native.load()
    s = _native.stream_ptr(st.dev)
    W = st.W
    ph, _, seed = st.drop
    if ph > 0:
        d = _dropout(lib, d, ph, seed, 0, s)
    demb, dge, dbe = layernorm_backward(d, emb_pre, W.emb_g, st.eps)
    dword = torch.zeros_like(W.word)
    dpos = torch.zeros_like(W.pos)
    dtype = torch.zeros_like(W.type)
    pad = st.model.embeddings.word_embeddings.padding_idx
    _native.check(lib.drt_embedding_bwd_types(st.ids.data_ptr(), _ptr(st.types), int(W.type.shape[0]),
                                              demb.data_ptr(), st.B, st.L, st.H, -1 if pad is None else int(pad),
                                              dword.data_ptr(), dpos.data_ptr(), dtype.data_ptr(), s),
                  "drt_embedding_bwd_types")
    e = "embeddings."
    return {e + "word_embeddings.weight": dword, e + "position_embeddings.weight": dpos,
            e + "token_type_embeddings.weight": dtype, e + "LayerNorm.weight": dge, e + "LayerNorm.bias": dbe}


def layer_forward(st: _Step, i: int, h):
    """One BertLayer (train-mode dropout as HF) -> (h_out, saved activations)."""
    lib = _native.load()
    dev = st.dev
    s = _native.stream_ptr(dev)
    ly = st.W.layers[i]
    B, L, H, heads = st.B, st.L, st.H, st.heads
    T = B * L
    ph, pa, seed = st.drop
    s_att, s_out1, s_out2 = dropout_sites(i)
    qkv = _lin(lib, h, ly["wqkv"], ly["bqkv"], torch.empty((T, 3 * H), dtype=torch.bfloat16, device=dev), stream=s)
    ctx = torch.empty((T, H), dtype=torch.bfloat16, device=dev)
    lse = torch.empty((B, heads, L), dtype=torch.float32, device=dev)
    # attention-dropout keep mask as bits (B * heads * L * L / 8 bytes): the backward reads it
    bits = torch.empty((B, heads, L, (L + 31) // 32), dtype=torch.int32, device=dev) if pa > 0 else None
    _native.check(lib.drt_attention_train_fwd_bits_bf16(qkv.data_ptr(), _ptr(st.mask), ctx.data_ptr(),
                                                        lse.data_ptr(), _ptr(bits), B, L, heads, H // heads, st.scale,
                                                        float(pa), seed, s_att, s),
                  "drt_attention_train_fwd_bits_bf16")
    # x1 = dropout(ctx Wo^T + bo) + h, dropout in the GEMM epilogue
    x1 = _lin(lib, ctx, ly["wo"], ly["bo"], torch.empty_like(h), resid=h, stream=s,
              drop=(ph, seed, s_out1) if ph > 0 else None)
    h1 = _layernorm(lib, x1, ly["g1"], ly["b1"], st.eps, s)
    # f = GELU(fpre), fpre = h1 Wi^T + bi: both from the one GEMM epilogue
    fpre = torch.empty((T, ly["wi"].shape[0]), dtype=torch.bfloat16, device=dev)
    f = _lin(lib, h1, ly["wi"], ly["bi"], torch.empty_like(fpre), gelu=True, stream=s, pre_out=fpre)
    # x2 = dropout(f Wf^T + bf) + h1
    x2 = _lin(lib, f, ly["wf"], ly["bf"], torch.empty_like(h), resid=h1, stream=s,
              drop=(ph, seed, s_out2) if ph > 0 else None)
    h2 = _layernorm(lib, x2, ly["g2"], ly["b2"], st.eps, s)
    return h2, (h, qkv, ctx, lse, bits, x1, h1, fpre, f, x2)


def layer_backward(st: _Step, i: int, saved, d) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """d h_in and the fp32 gradients of layer i's parameters (HF names) for d h_out."""
    lib = _native.load()
    s = _native.stream_ptr(st.dev)
    h, qkv, ctx, lse, bits, x1, h1, fpre, f, x2 = saved
    ly = st.W.layers[i]
    H, heads, eps = st.H, st.heads, st.eps
    ph, pa, seed = st.drop
    p = f"encoder.layer.{i}."
    s_att, s_out1, s_out2 = dropout_sites(i)
    # LN backward also emits the dropped gradient entering FFN2; FFN2's dgrad applies the GELU
    # backward in its epilogue (-> d fpre)
    # (the LayerNorm backwards also return the column sums of what they hand down: the dense
    # biases' gradients, without a pass over dy2 / dy1)
    if ph > 0:
        dx2, dg2, db2, dy2, sum2 = layernorm_backward(d, x2, ly["g2"], eps, drop=(ph, seed, s_out2), want_sum=True)
    else:
        dx2, dg2, db2, sum2 = layernorm_backward(d, x2, ly["g2"], eps, want_sum=True)
        dy2 = dx2
    dbi = torch.empty(fpre.shape[1], dtype=torch.float32, device=st.dev)   # from FFN2's dgrad epilogue
    dfpre, dwf, dbf = linear_backward(dy2, f, ly["wf_t"], gelu_pre=fpre, db=sum2, dx_colsum=dbi)
    dh1, dwi, dbi = linear_backward(dfpre, h1, ly["wi_t"], resid=dx2, db=dbi)
    if ph > 0:
        dx1, dg1, db1, dy1, sum1 = layernorm_backward(dh1, x1, ly["g1"], eps, drop=(ph, seed, s_out1), want_sum=True)
    else:
        dx1, dg1, db1, sum1 = layernorm_backward(dh1, x1, ly["g1"], eps, want_sum=True)
        dy1 = dx1
    dctx, dwo, dbo = linear_backward(dy1, ctx, ly["wo_t"], db=sum1)
    dqkv = torch.empty_like(qkv)
    # the attention backward also leaves per-sequence column sums of dQKV: the q / k / v bias
    # gradients without a pass over dQKV
    dbqkv = torch.empty(3 * H, dtype=torch.float32, device=st.dev)
    nb = int(lib.drt_attention_train_bwd_bias_workspace(st.B, heads, H // heads))
    ws = torch.empty((nb + 3) // 4, dtype=torch.float32, device=st.dev)
    _native.check(lib.drt_attention_train_bwd_bias_bf16(qkv.data_ptr(), ctx.data_ptr(), dctx.data_ptr(),
                                                        lse.data_ptr(), _ptr(st.mask), _ptr(bits), dqkv.data_ptr(),
                                                        st.B, st.L, heads, H // heads, st.scale, float(pa), seed,
                                                        s_att, dbqkv.data_ptr(), ws.data_ptr(), nb, s),
                  "drt_attention_train_bwd_bias_bf16")
    d_in, dwqkv, dbqkv = linear_backward(dqkv, h, ly["wqkv_t"], resid=dx1, db=dbqkv)
    grads = {}
    grads[p + "output.LayerNorm.weight"], grads[p + "output.LayerNorm.bias"] = dg2, db2
    grads[p + "output.dense.weight"], grads[p + "output.dense.bias"] = dwf, dbf
    grads[p + "intermediate.dense.weight"], grads[p + "intermediate.dense.bias"] = dwi, dbi
    grads[p + "attention.output.LayerNorm.weight"], grads[p + "attention.output.LayerNorm.bias"] = dg1, db1
    grads[p + "attention.output.dense.weight"], grads[p + "attention.output.dense.bias"] = dwo, dbo
    for j, n in enumerate(("query", "key", "value")):
        grads[p + f"attention.self.{n}.weight"] = dwqkv[j * H:(j + 1) * H]
        grads[p + f"attention.self.{n}.bias"] = dbqkv[j * H:(j + 1) * H]
    return d_in, grads


# One autograd node per BertLayer (and one for the embeddings): each node's parameter gradients
# are handed to autograd (AccumulateGrad, so DDP's bucket hooks) as soon as THAT layer's backward
# is done, and DDP's gradient all-reduce of layer i overlaps the backward of layers i-1 .. 0
# (trainer.py:47-63 wraps the model in DDP).  The activation between nodes is the bf16 hidden
# state; all nodes of one pass share a _Step (weights snapshot, ids, mask, dropout seed).
def _grads_out(names, grads):
    return tuple(grads[n].to(torch.float32) if n in grads else None for n in names)


class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, st, names, *params):
        h, emb_pre = embed_forward(st)
        ctx.st, ctx.emb_pre, ctx.names = st, emb_pre, names
        return h

    @staticmethod
    def backward(ctx, d):
        grads = embed_backward(ctx.st, ctx.emb_pre, d.contiguous())
        ctx.emb_pre = None
        return (None, None, None) + _grads_out(ctx.names, grads)


class _LayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, st, i, names, *params):
        h2, saved = layer_forward(st, i, h)
        ctx.st, ctx.i, ctx.saved_acts, ctx.names = st, i, saved, names
        return h2

    @staticmethod
    def backward(ctx, d):
        d_in, grads = layer_backward(ctx.st, ctx.i, ctx.saved_acts, d.contiguous())
        ctx.saved_acts = None
        return (d_in, None, None, None) + _grads_out(ctx.names, grads)


def _param_groups(model):
    """(embedding names/params, [per-layer names/params]) in the HF naming."""
    named = dict(model.named_parameters())
    emb = [n for n in named if n.startswith("embeddings.")]
    layers = []
    for i in range(model.config.num_hidden_layers):
        pre = f"encoder.layer.{i}."
        layers.append([n for n in named if n.startswith(pre)])
    return named, emb, layers


def train_hidden(model, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor],
                 seed: Optional[int] = None, token_type_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
    """last_hidden_state fp32 [B, L, H] of ``model`` with the HIP tower backward attached (one autograd
    node per layer).  Dropout follows ``model.training`` and the config's probabilities (seed: torch
    CPU RNG)."""
    why = tower_supported(model)
    if why is not None:
        raise NotImplementedError(f"HIP training tower: {why}")
    dev = next(model.parameters()).device
    ids = input_ids.to(dev, torch.int64).contiguous()
    mask = attention_mask.to(dev, torch.int64).contiguous() if attention_mask is not None else None
    types = token_type_ids.to(dev, torch.int64).contiguous() if token_type_ids is not None else None
    if types is not None and (types.shape != ids.shape or model.config.type_vocab_size > 4):
        raise ValueError("HIP training tower: token_type_ids must match input_ids, type_vocab_size <= 4")
    B, L = ids.shape
    cfg = model.config
    lmax = min(MAX_TRAIN_SEQ, int(cfg.max_position_embeddings))
    if L > lmax:
        raise ValueError(f"HIP training tower: sequence length {L} > {lmax}")
    ph = float(cfg.hidden_dropout_prob) if model.training else 0.0
    pa = float(cfg.attention_probs_dropout_prob) if model.training else 0.0
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if (ph > 0 or pa > 0) else 0
    st = _Step(model, _Weights(model, dev), ids, mask, (ph, pa, seed), types)
    named, emb, layers = _param_groups(model)
    h = _EmbedFn.apply(ids, st, emb, *[named[n] for n in emb])
    for i, names in enumerate(layers):
        h = _LayerFn.apply(h, st, i, names, *[named[n] for n in names])
    return h.view(B, L, cfg.hidden_size).float()
