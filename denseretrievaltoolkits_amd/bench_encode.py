"""Encode leg of bench.py: passages encoded/sec of the bf16 BERT-base passage tower.

Config C2 (BASELINE.json configs[1]): DPR bert-base, 128-token passages.
Random-init BERT-base weights (no checkpoint offline), synthetic token ids in
the collator format; one step = DRModel.encode_passage of one batch
(embeddings -> 12 layers -> [CLS] pooling), all on the HIP kernels.
"""
from __future__ import annotations

import time

import torch

FLOP_PER_PASSAGE_L128 = 22.347e9   # linear 169.87 MFLOP/token + attention 4*L^2*768*12


def flops_per_seq(L, H=768, layers=12, inter=3072):
    lin = 2 * L * (H * 3 * H + H * H + 2 * H * inter) * layers
    att = 4 * L * L * H * layers
    return lin + att


def run(device, batch=512, L=128, steps=10, warmup=2):
    from transformers import BertConfig, BertModel
    from .model.encoder import HipBertEncoder
    from . import _native
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(m, device)
    del m
    g = torch.Generator(device=device)
    g.manual_seed(1)
    ids = torch.randint(1000, 30522, (batch, L), generator=g, device=device, dtype=torch.int64)
    ids[:, 0] = 101
    ids[:, -1] = 102
    mask = torch.ones((batch, L), dtype=torch.int64, device=device)
    lib = _native.load()
    for _ in range(warmup):
        enc.pool(enc(ids, mask), mask, "first")
    torch.cuda.synchronize()
    lib.drt_profile_enable(_native.PROF_GEMM, 1)
    t0 = time.perf_counter()
    for _ in range(steps):
        enc.pool(enc(ids, mask), mask, "first")
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    lib.drt_profile_enable(_native.PROF_GEMM, 0)
    tot = _native.ctypes.c_double(0)
    cnt = _native.c_i64(0)
    lib.drt_profile_read(_native.PROF_GEMM, _native.ctypes.byref(tot), _native.ctypes.byref(cnt))
    pps = steps * batch / el
    fl = flops_per_seq(L)
    gemm_flops = 2 * L * batch * (768 * 3 * 768 + 768 * 768 + 2 * 768 * 3072) * 12 * steps
    # per-launch event times only add up to GEMM time when one stream runs at a time; with the
    # two-stream split (HipBertEncoder.split_streams) they overlap the other half's kernels
    split = enc.split_streams and batch >= 2 and batch * L >= enc.split_min_tokens
    gemm_tf = gemm_flops / (tot.value * 1e-3) / 1e12 if tot.value > 0 and not split else None
    return {
        "metric": "passages encoded/sec (bf16 BERT-base, 128-token passages)",
        "value": round(pps, 1),
        "unit": "passages/s",
        "batch": batch, "seq_len": L, "steps": steps,
        "ms_per_step": round(el / steps * 1e3, 3),
        "roofline": {
            "bound": "mfma",
            "achieved": round(fl * pps / 1e12, 1),
            "peak": 2500.0,
            "unit": "TFLOP/s",
            "frac": round(fl * pps / 1e12 / 2500.0, 4),
            "flop_per_passage": fl,
            "gemm_only_tflops": round(gemm_tf, 1) if gemm_tf else None,
            "streams": 2 if split else 1,
        },
    }


def run_query_encode(device, batches=(8, 128), L=32, steps=50, warmup=3):
    """Query tower (C4: queries of 32 tokens, searched in batches of 128): DRModel.encode_query's
    HIP forward + [CLS] pooling, eager launches vs hipGraph replay (HipBertEncoder._replay), at a
    small interactive batch (8: host-bound when eager) and the search batch (128: GPU-bound)."""
    from transformers import BertConfig, BertModel
    from .model.encoder import HipBertEncoder
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(m, device)
    del m
    g = torch.Generator(device=device)
    g.manual_seed(4)
    fl = flops_per_seq(L)
    res = {"metric": f"queries encoded/sec (bf16 BERT-base query tower, {L} tokens)", "unit": "queries/s",
           "seq_len": L, "steps": steps}
    for batch in batches:
        ids = torch.randint(1000, 30522, (batch, L), generator=g, device=device, dtype=torch.int64)
        ids[:, 0] = 101
        ids[:, -1] = 102
        mask = torch.ones((batch, L), dtype=torch.int64, device=device)
        r = {}
        for name, graphs in (("eager", False), ("graph", True)):
            enc.graphs = graphs
            for _ in range(warmup):
                enc.pool(enc(ids, mask), mask, "first")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                enc.pool(enc(ids, mask), mask, "first")
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            r[name] = round(steps * batch / el, 1)
            r[name + "_ms_per_batch"] = round(el / steps * 1e3, 4)
        r["mfma_frac"] = round(fl * r["graph"] / 1e12 / 2500.0, 4)
        res[f"b{batch}"] = r
    res["value"] = res[f"b{batches[-1]}"]["eager"]   # the default path (encoder.graphs = False)
    return res


def run_rerank(device, pairs=1000, q_len=32, p_len=128, steps=3, warmup=1):
    """Config C5 (BASELINE.json configs[4]): cross-encoder rerank of the top-1000
    candidates of one query per step (RRModel.encode, DRT/model/reranker.py:111-130):
    1000 pairs [CLS] q [SEP] p [SEP] of L = q_len + p_len = 160 tokens through the bf16
    BERT-base tower, [CLS] pooling, LinearHead(768 -> 1)."""
    from transformers import BertConfig, BertModel
    from .model.encoder import HipBertEncoder, linear_head
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(m, device)
    del m
    L = q_len + p_len
    g = torch.Generator(device=device)
    g.manual_seed(2)
    ids = torch.randint(1000, 30522, (pairs, L), generator=g, device=device, dtype=torch.int64)
    ids[:, 0] = 101
    ids[:, q_len - 1] = 102
    ids[:, -1] = 102
    mask = torch.ones((pairs, L), dtype=torch.int64, device=device)
    head_w = (0.02 * torch.randn((1, 768), generator=g, device=device)).to(torch.bfloat16)

    def step():
        _, rb = enc.pool(enc(ids, mask), mask, "first", want_bf16=True)
        return linear_head(rb, head_w)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    qps = steps / el
    fl = flops_per_seq(L) * pairs
    return {
        "metric": f"queries/sec reranked (top-{pairs} pairs per query, L={L}, bf16 BERT-base cross-encoder)",
        "value": round(qps, 2), "unit": "queries/s", "pairs_per_query": pairs, "seq_len": L, "steps": steps,
        "ms_per_step": round(el / steps * 1e3, 3),
        "roofline": {"bound": "mfma", "achieved": round(fl * qps / 1e12, 1), "peak": 2500.0, "unit": "TFLOP/s",
                     "frac": round(fl * qps / 1e12 / 2500.0, 4), "flop_per_pair": flops_per_seq(L)},
    }


def run_train_scores(device, bq=512, d=768, n_passages=(2, 8), steps=20, warmup=3):
    """Config C3 (BASELINE.json configs[2]): the in-batch-negative score matrix of
    DRModel.forward (DRT/model/biencoder.py:107-119) at batch 512: scores = q . p^T
    [512, 512 n], CrossEntropy(mean) with target i * n, and its backward (dq, dp),
    fp32 end to end on the HIP op (torch.ops.drt.score_ce_fwd, score_ce.py), next to torch's fp32
    matmul + cross_entropy + autograd on the same device."""
    from .score_ce import score_ce
    g = torch.Generator(device=device)
    g.manual_seed(3)
    res = {"metric": "in-batch-negative score+CE forward+backward, ms per step (fp32)", "batch": bq, "dim": d}
    for n in n_passages:
        q = torch.randn((bq, d), generator=g, device=device).requires_grad_(True)
        p = torch.randn((bq * n, d), generator=g, device=device).requires_grad_(True)
        tgt = torch.arange(bq, device=device) * n

        def ours():
            loss, _ = score_ce(q, p, n, 1.0)
            loss.backward()

        def ref():
            s = q @ p.T
            torch.nn.functional.cross_entropy(s, tgt).backward()

        out = {}
        for name, fn in (("hip", ours), ("torch", ref)):
            for _ in range(warmup):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                fn()
            torch.cuda.synchronize()
            out[name + "_ms"] = round((time.perf_counter() - t0) / steps * 1e3, 4)
        # device time of the same step: captured once in a hipGraph (torch.cuda.graph) and replayed,
        # so host-side autograd / Python overhead (which dominates both eager timings) drops out
        for name, fn in (("hip", ours), ("torch", ref)):
            try:
                side = torch.cuda.Stream(device)
                side.wait_stream(torch.cuda.current_stream(device))
                with torch.cuda.stream(side):
                    for _ in range(warmup):
                        fn()
                torch.cuda.current_stream(device).wait_stream(side)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    fn()
                graph.replay()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps * 5):
                    graph.replay()
                torch.cuda.synchronize()
                out[name + "_graph_ms"] = round((time.perf_counter() - t0) / (steps * 5) * 1e3, 4)
                del graph
            except Exception as e:  # report, keep the bench line
                out[name + "_graph_error"] = f"{type(e).__name__}: {e}"[:200]
        fl = 6 * bq * bq * n * d
        out["flop"] = fl
        out["hip_tflops"] = round(fl / (out["hip_ms"] * 1e-3) / 1e12, 2)
        if "hip_graph_ms" in out:
            out["hip_graph_tflops"] = round(fl / (out["hip_graph_ms"] * 1e-3) / 1e12, 2)
        res[f"n{n}"] = out
    return res


def run_train_step(device, bq=512, n=2, q_len=32, p_len=128, steps=3, warmup=1):
    """Config C3 end to end: one in-batch-negative training step of DRModel.forward (query tower on
    512 x 32 tokens, passage tower on 1024 x 128 tokens, score matrix + CE, backward into every
    tower parameter; DRT/trainer/trainer.py:113-133) on BERT-base (random init):
    the HIP training tower (bf16 activations, model/train_tower.py) vs the HF module under torch
    fp32 autograd on the same device, both with HF's default dropout (0.1 hidden / 0.1 attention:
    HF's own masks vs the tower's hash masks).  Optimizer update excluded (identical for both)."""
    from types import SimpleNamespace
    from transformers import BertConfig, BertModel
    from .model.biencoder import DRModel
    torch.manual_seed(0)
    lm = BertModel(BertConfig(), add_pooling_layer=False).to(device).train()
    m = DRModel(lm_q=lm, lm_p=lm, pooling="first", data_args=SimpleNamespace(train_n_passages=n),
                train_args=SimpleNamespace(negatives_x_device=False)).train()
    g = torch.Generator(device=device)
    g.manual_seed(6)

    def batch(b, L):
        ids = torch.randint(1000, 30522, (b, L), generator=g, device=device, dtype=torch.int64)
        ids[:, 0] = 101
        ids[:, -1] = 102
        return {"input_ids": ids, "attention_mask": torch.ones((b, L), dtype=torch.int64, device=device)}

    qry, psg = batch(bq, q_len), batch(bq * n, p_len)
    fl = 3 * (bq * flops_per_seq(q_len) + bq * n * flops_per_seq(p_len))
    res = {"metric": "in-batch-negative training step (fwd + bwd of both towers + score/CE), ms",
           "batch": bq, "train_n_passages": n, "q_len": q_len, "p_len": p_len, "flop_per_step": fl}
    # torch_bf16_autocast: the same HF module under torch.autocast(bf16) (hipBLASLt GEMMs + sdpa), the
    # like-for-like arithmetic baseline for the bf16 HIP tower (the reference itself is fp32)
    for name, hip, amp in (("hip", True, False), ("torch_fp32", False, False), ("torch_bf16_autocast", False, True)):
        m.hip_train = hip

        def step():
            lm.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                loss = m(query=qry, passage=psg).loss
            loss.backward()

        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        res[name + "_ms"] = round(ms, 2)
        res[name + "_tflops"] = round(fl / (ms * 1e-3) / 1e12, 1)
    res["speedup"] = round(res["torch_fp32_ms"] / res["hip_ms"], 2)
    res["speedup_vs_bf16_autocast"] = round(res["torch_bf16_autocast_ms"] / res["hip_ms"], 2)
    res["mfma_frac"] = round(res["hip_tflops"] / 2500.0, 4)
    return res
