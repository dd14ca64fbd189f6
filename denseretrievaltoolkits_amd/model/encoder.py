"""BERT encoder forward on the HIP kernels (bf16 storage, fp32 accumulation).

Replaces the third-party HF ``BertModel.forward`` that ``DRModel.encode``
calls (DRT/model/biencoder.py:137; transformers modeling_bert.py:620-686) for
inference: embeddings + LayerNorm, then per layer

    qkv  = linear(h, Wqkv)                        (Q | K | V fused, bf16)
    ctx  = attention(qkv, key-padding mask)       (fused MFMA kernel)
    x    = linear(ctx, Wo) + bo + h               (fp32 sum, stored bf16)
    h    = layernorm(x)                           (fp32 statistics, bf16)
    f    = gelu(linear(h, W1) + b1)               (bf16)
    x    = linear(f, W2) + b2 + h                 (fp32 sum, stored bf16)
    h    = layernorm(x)

The pre-LayerNorm sums ``x`` are rounded once to bf16 (``presum="bf16"``, the
default): it halves the epilogue's store and the LayerNorm's load (≈ 5 % of
the forward); ``presum="fp32"`` keeps them fp32 (A/B and tests).

Weights are snapshotted from the HF module (bf16 copies of the linears,
fp32 embeddings / biases / LayerNorm) and re-snapshotted automatically when
the source parameters change (torch bumps ``Tensor._version`` on in-place
optimizer updates).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from .. import _native

POOL_MODES = {"first": 0, "mean": 1, "max": 2}


@dataclass
class BertShape:
    hidden: int
    layers: int
    heads: int
    intermediate: int
    eps: float
    act: str

    @classmethod
    def from_config(cls, cfg) -> "BertShape":
        return cls(cfg.hidden_size, cfg.num_hidden_layers, cfg.num_attention_heads, cfg.intermediate_size,
                   float(cfg.layer_norm_eps), str(cfg.hidden_act))


def _check_supported(shape: BertShape):
    if shape.hidden % 256 or shape.hidden > 1024:
        raise ValueError(f"hidden size {shape.hidden} unsupported (multiple of 256, <= 1024)")
    if shape.hidden // shape.heads != 64:
        raise ValueError("head_dim must be 64")
    if shape.intermediate % 64:
        raise ValueError("intermediate size must be a multiple of 64")
    if shape.act not in ("gelu", "gelu_new") and shape.act != "gelu":
        raise ValueError(f"activation {shape.act} unsupported (erf GELU only)")
    if shape.act != "gelu":
        raise ValueError("only erf GELU ('gelu') is implemented")


class HipBertEncoder:
    """Inference forward of a BERT-family encoder on gfx950 kernels."""

    def __init__(self, shape: BertShape, state: Dict[str, torch.Tensor], device: torch.device,
                 prefix: str = "", presum: str = "bf16"):
        _check_supported(shape)
        if presum not in ("bf16", "fp32"):
            raise ValueError(f"presum must be 'bf16' or 'fp32', got {presum!r}")
        self.presum = presum
        # hipGraph replay for B * L <= graph_max_tokens: off by default -- measured no gain
        # (bench query_encode: batch 8 and 128 are GPU-bound, the replay adds input/output copies)
        self.graphs = False
        self.graph_max_tokens = 16384
        self.graph_cache_size = 8
        self._graph_cache = {}
        self.split_streams = True       # two halves on two streams from split_min_tokens up
        self.fuse_ln = True             # dense + residual + LayerNorm in one call (_lin_ln)
        # from 8192 tokens: 256 x 32-token queries 2.47 -> 2.06 ms, 512 x 32 3.81 -> 3.74 (4096 tokens:
        # slower, 1.36 -> 1.50; tools/qenc_split_ab.py, profiles/r03zc_qenc_split_ab.log)
        self.split_min_tokens = 8192
        self._streams = None
        self._ws_plan = {}
        self._ws = None
        self.shape = shape
        self.device = device
        self.lib = _native.load()
        self._load(state, prefix)

    # -- weights --------------------------------------------------------
    def _load(self, sd: Dict[str, torch.Tensor], prefix: str):
        dev = self.device

        def f32(name):
            return sd[prefix + name].detach().to(dev, torch.float32).contiguous()

        def b16(name):
            return sd[prefix + name].detach().to(dev, torch.float32).to(torch.bfloat16).contiguous()

        self.word = f32("embeddings.word_embeddings.weight")
        self.pos = f32("embeddings.position_embeddings.weight")
        self.type = f32("embeddings.token_type_embeddings.weight")
        self.emb_g = f32("embeddings.LayerNorm.weight")
        self.emb_b = f32("embeddings.LayerNorm.bias")
        self.layers = []
        for i in range(self.shape.layers):
            p = f"encoder.layer.{i}."
            wqkv = torch.cat([sd[prefix + p + f"attention.self.{n}.weight"].detach().float()
                              for n in ("query", "key", "value")], 0)
            bqkv = torch.cat([sd[prefix + p + f"attention.self.{n}.bias"].detach().float()
                              for n in ("query", "key", "value")], 0)
            self.layers.append(dict(
                wqkv=wqkv.to(dev).to(torch.bfloat16).contiguous(),
                bqkv=bqkv.to(dev).contiguous(),
                wo=b16(p + "attention.output.dense.weight"), bo=f32(p + "attention.output.dense.bias"),
                g1=f32(p + "attention.output.LayerNorm.weight"), b1=f32(p + "attention.output.LayerNorm.bias"),
                wi=b16(p + "intermediate.dense.weight"), bi=f32(p + "intermediate.dense.bias"),
                wf=b16(p + "output.dense.weight"), bf=f32(p + "output.dense.bias"),
                g2=f32(p + "output.LayerNorm.weight"), b2=f32(p + "output.LayerNorm.bias"),
            ))

    @classmethod
    def from_hf(cls, model, device, presum: str = "bf16") -> "HipBertEncoder":
        return cls(BertShape.from_config(model.config), dict(model.state_dict()), torch.device(device),
                   presum=presum)

    # -- forward --------------------------------------------------------
    def _lin(self, x, w, b, out, resid=None, gelu=False):
        m, k = x.shape
        n = w.shape[0]
        flags = (1 if gelu else 0) | (2 if out.dtype == torch.float32 else 0)
        ws = self._ws
        _native.check(self.lib.drt_linear_bf16_ws(x.data_ptr(), w.data_ptr(), b.data_ptr() if b is not None else None,
                                                  resid.data_ptr() if resid is not None else None, out.data_ptr(),
                                                  m, n, k, flags, ws.data_ptr() if ws is not None else None,
                                                  ws.numel() * 4 if ws is not None else 0, self.stream),
                      "drt_linear_bf16_ws")
        return out

    def _lin_ln(self, x, w, b, h, g, beta, x32, ln):
        """h = LayerNorm(x w^T + b + h) (BertSelfOutput / BertOutput, modeling_bert.py:282-352).  bf16
        pre-LayerNorm sums: one call that finishes a split-K GEMM and the LayerNorm in a single launch
        when the split plan applies (query-sized batches), bit-identical to linear + LayerNorm."""
        m, k = x.shape
        n = w.shape[0]
        T, H = h.shape
        if self.fuse_ln and x32.dtype == torch.bfloat16 and H % 256 == 0 and H <= 1024:
            ws = self._ws
            _native.check(self.lib.drt_linear_ln_bf16_ws(
                x.data_ptr(), w.data_ptr(), b.data_ptr(), h.data_ptr(), g.data_ptr(), beta.data_ptr(),
                self.shape.eps, x32.data_ptr(), h.data_ptr(), m, n, k, ws.data_ptr() if ws is not None else None,
                ws.numel() * 4 if ws is not None else 0, self.stream), "drt_linear_ln_bf16_ws")
            return h
        self._lin(x, w, b, x32, resid=h)
        _native.check(ln(x32.data_ptr(), T, H, g.data_ptr(), beta.data_ptr(), self.shape.eps, h.data_ptr(),
                         self.stream), "drt_layernorm")
        return h

    def _ws_bytes(self, T: int) -> int:
        """Split-K scratch for this token count (small batches only; 0 at encode sizes)."""
        nb = self._ws_plan.get(T)
        if nb is None:
            H, I = self.shape.hidden, self.shape.intermediate
            nb = max(int(self.lib.drt_linear_workspace(T, n, k)) for n, k in ((3 * H, H), (H, H), (I, H), (H, I)))
            self._ws_plan[T] = nb
        return nb

    def forward(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                token_type_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
        """last_hidden_state [B, L, H] bf16."""
        dev = self.device
        ids = input_ids.to(dev, torch.int64).contiguous()
        B, L = ids.shape
        if L > self.pos.shape[0]:
            raise ValueError(f"sequence length {L} exceeds max_position_embeddings {self.pos.shape[0]}")
        mask = attention_mask.to(dev, torch.int64).contiguous() if attention_mask is not None else None
        tt = token_type_ids.to(dev, torch.int64).contiguous() if token_type_ids is not None else None
        if (self.graphs and 0 < B * L <= self.graph_max_tokens
                and not torch.cuda.is_current_stream_capturing()):
            return self._replay(ids, mask, tt)
        if (self.split_streams and B >= 2 and B * L >= self.split_min_tokens
                and not torch.cuda.is_current_stream_capturing()):
            return self._run_halves(ids, mask, tt)
        return self._run(ids, mask, tt)

    # -- two halves on two streams ----------------------------------------
    # Large batches run as two independent halves on two HIP streams: one half's memory-bound
    # kernels (attention, LayerNorm) and GEMM tails overlap the other half's GEMMs (+4.4 % on the
    # encode leg, tools/enc_streams.py).  Same kernels per half -> bit-identical to one pass.
    def _run_halves(self, ids, mask, tt):
        dev = self.device
        B, L = ids.shape
        H = self.shape.hidden
        out = torch.empty((B * L, H), dtype=torch.bfloat16, device=dev)
        cur = torch.cuda.current_stream(dev)
        if self._streams is None:
            self._streams = [torch.cuda.Stream(dev) for _ in range(2)]
        half = B // 2
        for i, (a, b) in enumerate(((0, half), (half, B))):
            st = self._streams[i]
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                self._run(ids[a:b], mask[a:b] if mask is not None else None, tt[a:b] if tt is not None else None,
                          out=out[a * L:b * L])
            out.record_stream(st)
        for st in self._streams:
            cur.wait_stream(st)
        return out.view(B, L, H)

    # -- hipGraph replay ------------------------------------------------
    # Small batches (queries: 128 x 32 tokens) are host-bound: 1 + 7 x layers launches through
    # ctypes cost more host time than the GPU needs.  Each (B, L, mask?, types?) shape is
    # captured once into a hipGraph (torch.cuda.graph on the launch stream) and replayed: one
    # host call per forward.  Inputs are copied into the graph's static buffers; the output is
    # a copy of the graph's static output (the next replay overwrites it).  A new encoder is
    # built whenever the weights change (biencoder._hip_encoder), which drops its graphs.
    def _replay(self, ids, mask, tt):
        key = (tuple(ids.shape), mask is not None, tt is not None)
        ent = self._graph_cache.get(key)
        if ent is None:
            dev = self.device
            si = ids.clone()
            sm = mask.clone() if mask is not None else None
            st = tt.clone() if tt is not None else None
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):     # eager warm-up: one-time kernel attributes, allocator
                self._run(si, sm, st)
            torch.cuda.current_stream(dev).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = self._run(si, sm, st)
            if len(self._graph_cache) >= self.graph_cache_size:
                self._graph_cache.pop(next(iter(self._graph_cache)))
            ent = self._graph_cache[key] = (g, si, sm, st, out)
        g, si, sm, st, out = ent
        si.copy_(ids)
        if sm is not None:
            sm.copy_(mask)
        if st is not None:
            st.copy_(tt)
        g.replay()
        return out.clone()

    def _run(self, ids, mask, tt, out=None):
        sh = self.shape
        dev = self.device
        B, L = ids.shape
        H, T = sh.hidden, B * L
        self.stream = _native.stream_ptr(dev)
        h = out if out is not None else torch.empty((T, H), dtype=torch.bfloat16, device=dev)
        _native.check(self.lib.drt_embed_ln(ids.data_ptr(), tt.data_ptr() if tt is not None else None, B, L,
                                            self.word.data_ptr(), self.pos.data_ptr(), self.type.data_ptr(),
                                            self.emb_g.data_ptr(), self.emb_b.data_ptr(), sh.eps, H, h.data_ptr(),
                                            self.stream), "drt_embed_ln")
        qkv = torch.empty((T, 3 * H), dtype=torch.bfloat16, device=dev)
        ctx = torch.empty((T, H), dtype=torch.bfloat16, device=dev)
        f32 = self.presum == "fp32"
        x32 = torch.empty((T, H), dtype=torch.float32 if f32 else torch.bfloat16, device=dev)
        ln = self.lib.drt_layernorm_f32_bf16 if f32 else self.lib.drt_layernorm_bf16
        ffn = torch.empty((T, sh.intermediate), dtype=torch.bfloat16, device=dev)
        nb = self._ws_bytes(T)
        self._ws = torch.empty((nb + 3) // 4, dtype=torch.float32, device=dev) if nb else None
        scale = 1.0 / math.sqrt(H // sh.heads)
        for ly in self.layers:
            self._lin(h, ly["wqkv"], ly["bqkv"], qkv)
            _native.check(self.lib.drt_attention_bf16(qkv.data_ptr(), mask.data_ptr() if mask is not None else None,
                                                      ctx.data_ptr(), B, L, sh.heads, H // sh.heads, scale,
                                                      self.stream), "drt_attention_bf16")
            self._lin_ln(ctx, ly["wo"], ly["bo"], h, ly["g1"], ly["b1"], x32, ln)
            self._lin(h, ly["wi"], ly["bi"], ffn, gelu=True)
            self._lin_ln(ffn, ly["wf"], ly["bf"], h, ly["g2"], ly["b2"], x32, ln)
        return h.view(B, L, H)

    __call__ = forward

    def pool(self, hidden: torch.Tensor, attention_mask: Optional[torch.Tensor], pooling: str,
             want_bf16: bool = False):
        """reps fp32 [B, H] (and optional bf16 copy) with the reference's pooling semantics."""
        if pooling not in POOL_MODES:
            raise ValueError("Unknown pooling type: {}".format(pooling))
        B, L, H = hidden.shape
        dev = hidden.device
        mask = attention_mask.to(dev, torch.int64).contiguous() if attention_mask is not None else None
        reps = torch.empty((B, H), dtype=torch.float32, device=dev)
        rb = torch.empty((B, H), dtype=torch.bfloat16, device=dev) if want_bf16 else None
        _native.check(self.lib.drt_pool_bf16(hidden.data_ptr(), mask.data_ptr() if mask is not None else None,
                                             B, L, H, POOL_MODES[pooling], reps.data_ptr(),
                                             rb.data_ptr() if rb is not None else None, _native.stream_ptr(dev)),
                      "drt_pool_bf16")
        return reps, rb


def l2_normalize_(reps: torch.Tensor, want_bf16: bool = False):
    lib = _native.load()
    reps = reps.contiguous()
    B, H = reps.shape
    rb = torch.empty((B, H), dtype=torch.bfloat16, device=reps.device) if want_bf16 else None
    _native.check(lib.drt_l2_normalize_f32(reps.data_ptr(), B, H, rb.data_ptr() if rb is not None else None,
                                           _native.stream_ptr(reps.device)), "drt_l2_normalize_f32")
    return reps, rb


def linear_head(reps_bf16: torch.Tensor, weight_bf16: torch.Tensor) -> torch.Tensor:
    """LinearHead.forward (DRT/model/linear.py:22-23): reps @ W^T, no bias, fp32 out."""
    lib = _native.load()
    B, K = reps_bf16.shape
    N = weight_bf16.shape[0]
    out = torch.empty((B, N), dtype=torch.float32, device=reps_bf16.device)
    if K % 64:
        raise ValueError("head input dim must be a multiple of 64")
    _native.check(lib.drt_linear_bf16(reps_bf16.data_ptr(), weight_bf16.data_ptr(), None, None, out.data_ptr(),
                                      B, N, K, 2, _native.stream_ptr(reps_bf16.device)), "drt_linear_bf16")
    return out
