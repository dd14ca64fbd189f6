"""Encode leg A/B: how the independent parts of a batch share the GPU (bf16 BERT-base, L = 128).

  base      HipBertEncoder as shipped: two halves on two streams, each issued whole (lockstep)
  lag_attn  two halves, the second half's layer i starts after the first half's QKV + attention of
            layer i (event): the halves run different GEMMs at the same time, so their epilogue
            write bursts and LDS-DMA phases fall apart
  lag_ffn1  as lag_attn, the lag point after the first half's FFN1
  quarters  four quarter batches on four streams, issued whole
  one       one pass, no split
Outputs of every variant are checked equal to `base` (same kernels per part).
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(rounds=3, steps=8, B=512):
    import math
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd import _native
    from denseretrievaltoolkits_amd.model.encoder import HipBertEncoder
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(m, dev)
    del m
    L = 128
    sh = enc.shape
    H = sh.hidden
    ids = torch.randint(1000, 30522, (B, L), device=dev)
    mask = torch.ones((B, L), dtype=torch.int64, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    out = torch.empty((B * L, H), dtype=torch.bfloat16, device=dev)

    def bufs(T):
        return dict(qkv=torch.empty((T, 3 * H), dtype=torch.bfloat16, device=dev),
                    ctx=torch.empty((T, H), dtype=torch.bfloat16, device=dev),
                    x32=torch.empty((T, H), dtype=torch.bfloat16, device=dev),
                    ffn=torch.empty((T, sh.intermediate), dtype=torch.bfloat16, device=dev))

    half_bufs = [bufs(B // 2 * L) for _ in range(2)]
    scale = 1.0 / math.sqrt(H // sh.heads)

    def lagged(lag_after):
        """two halves; stream 1's op j of layer i waits for stream 0's event after op lag_after of
        layer i (ops: 0 QKV, 1 attention, 2 O-proj+LN, 3 FFN1, 4 FFN2+LN)."""
        cur = torch.cuda.current_stream(dev)
        half = B // 2
        parts = [(0, half), (half, B)]
        hs = []
        for i, (a, b) in enumerate(parts):
            st = streams[i]
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                enc._ws = None
                enc.stream = _native.stream_ptr(dev)
                h = out[a * L:b * L]
                _native.check(enc.lib.drt_embed_ln(ids[a:b].data_ptr(), None, b - a, L, enc.word.data_ptr(),
                                                   enc.pos.data_ptr(), enc.type.data_ptr(), enc.emb_g.data_ptr(),
                                                   enc.emb_b.data_ptr(), sh.eps, H, h.data_ptr(), enc.stream),
                              "embed")
                hs.append(h)
        evs = [[torch.cuda.Event() for _ in range(5)] for _ in enc.layers]
        for li, ly in enumerate(enc.layers):
            for i, (a, b) in enumerate(parts):
                st = streams[i]
                bf = half_bufs[i]
                h = hs[i]
                with torch.cuda.stream(st):
                    enc.stream = _native.stream_ptr(dev)
                    enc._ws = None
                    ops = [
                        lambda: enc._lin(h, ly["wqkv"], ly["bqkv"], bf["qkv"]),
                        lambda: _native.check(enc.lib.drt_attention_bf16(
                            bf["qkv"].data_ptr(), mask[a:b].data_ptr(), bf["ctx"].data_ptr(), b - a, L, sh.heads,
                            H // sh.heads, scale, enc.stream), "attn"),
                        lambda: enc._lin_ln(bf["ctx"], ly["wo"], ly["bo"], h, ly["g1"], ly["b1"], bf["x32"],
                                            enc.lib.drt_layernorm_bf16),
                        lambda: enc._lin(h, ly["wi"], ly["bi"], bf["ffn"], gelu=True),
                        lambda: enc._lin_ln(bf["ffn"], ly["wf"], ly["bf"], h, ly["g2"], ly["b2"], bf["x32"],
                                            enc.lib.drt_layernorm_bf16),
                    ]
                    for j, op in enumerate(ops):
                        if i == 1 and j == 0 and lag_after is not None:
                            st.wait_event(evs[li][lag_after])
                        op()
                        if i == 0:
                            evs[li][j].record(st)
        for st in streams[:2]:
            cur.wait_stream(st)
        return out.view(B, L, H)

    def parts_whole(n):
        cur = torch.cuda.current_stream(dev)
        step = B // n
        for i in range(n):
            st = streams[i]
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                enc._run(ids[i * step:(i + 1) * step], mask[i * step:(i + 1) * step], None,
                         out=out[i * step * L:(i + 1) * step * L])
            out.record_stream(st)
        for st in streams[:n]:
            cur.wait_stream(st)
        return out.view(B, L, H)

    def one():
        enc.split_streams = False
        r = enc(ids, mask)
        enc.split_streams = True
        return r

    variants = {
        "base": lambda: enc(ids, mask),
        "lag_attn": lambda: lagged(1),
        "lag_oproj": lambda: lagged(2),
        "lag_ffn1": lambda: lagged(3),
        "quarters": lambda: parts_whole(4),
        "one": one,
    }
    ref = variants["base"]().clone()
    torch.cuda.synchronize()
    same = {}
    for name, fn in variants.items():
        r = fn()
        torch.cuda.synchronize()
        same[name] = bool(torch.equal(r, ref))
    res = {}
    for _ in range(rounds):
        for name, fn in variants.items():
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                fn()
            torch.cuda.synchronize()
            res.setdefault(name, []).append(round(steps * B / (time.perf_counter() - t0), 1))
    print(json.dumps({"B": B, "median_passages_per_s": {k: sorted(v)[len(v) // 2] for k, v in res.items()},
                      "rounds": res, "bit_identical_to_base": same}))


if __name__ == "__main__":
    main(B=int(sys.argv[1]) if len(sys.argv) > 1 else 512)
