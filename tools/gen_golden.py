#!/usr/bin/env python3
"""Generate golden fixtures from the REFERENCE implementation (run in the survey
container only; /root/reference does not exist on the GPU box).

    PYTHONPATH=/root/reference HF_HUB_OFFLINE=1 python tools/gen_golden.py

Imports the reference's own modules (DRT.model.biencoder.DRModel,
DRT.model.utils.merge_retrieval_results_by_score,
DRT.trainer.losses.SimpleContrastiveLoss, DRT.evaluator.metrics.get_metrics)
and records inputs + outputs as small .npz / .json fixtures under tests/golden/.
Model weights are NOT stored: they are regenerated from
oracle/bert_weights.param_value(seed, name, shape) on both sides.
"""
from __future__ import annotations

import json
import os
import sys
from types import SimpleNamespace

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.path.join(REPO, "tests", "golden")

from oracle import bert_weights as bw  # noqa: E402


def _ref():
    import DRT.evaluator.metrics as ref_metrics
    import DRT.model.biencoder as ref_bi
    import DRT.model.linear as ref_linear
    import DRT.model.utils as ref_utils
    import DRT.trainer.losses as ref_losses
    assert os.path.abspath(ref_bi.__file__).startswith("/root/reference"), ref_bi.__file__
    return ref_bi, ref_linear, ref_utils, ref_losses, ref_metrics


def gen_encode(ref_bi, ref_linear, layers, seed, variants, B, L, tag):
    from transformers import BertModel
    torch.manual_seed(0)
    lm = BertModel(bw.bert_config(layers=layers), add_pooling_layer=False).eval()
    bw.init_model_(lm, seed)
    ids, mask = bw.token_batch(B, L, seed=seed + 17)
    out = {"input_ids": ids, "attention_mask": mask}
    for pooling, normalize, head in variants:
        h = None
        if head:
            h = ref_linear.LinearHead(768, 768)
            with torch.no_grad():
                h.linear.weight.copy_(torch.from_numpy(bw.param_value(seed, "head.linear.weight", (768, 768))))
        model = ref_bi.DRModelForInference(lm_q=lm, lm_p=lm, tied=True, pooling=pooling, head_q=h, head_p=h,
                                           normalize=normalize).eval()
        with torch.no_grad():
            res = model(passage={"input_ids": torch.from_numpy(ids), "attention_mask": torch.from_numpy(mask)})
        out[f"reps_{pooling}_{int(normalize)}_{int(head)}"] = res.p_reps.numpy()
    np.savez_compressed(os.path.join(OUT, f"encode_{tag}.npz"), layers=layers, seed=seed, **out)


def gen_loss(ref_bi, ref_losses):
    rng = np.random.default_rng(123)
    cases = {}
    for name, (bq, n, d) in {"n2": (8, 2, 768), "n8": (4, 8, 64)}.items():
        q = rng.standard_normal((bq, d)).astype(np.float32)
        p = rng.standard_normal((bq * n, d)).astype(np.float32)
        qt = torch.from_numpy(q).requires_grad_(True)
        pt = torch.from_numpy(p).requires_grad_(True)
        loss = ref_losses.SimpleContrastiveLoss()(qt, pt)
        loss.backward()
        # DRModel.forward's own score matrix + CE on the same reps (biencoder.py:107-116)
        scores = torch.matmul(torch.from_numpy(q), torch.from_numpy(p).T).numpy()
        cases.update({f"{name}_q": q, f"{name}_p": p, f"{name}_loss": np.float32(loss.item()),
                      f"{name}_dq": qt.grad.numpy(), f"{name}_dp": pt.grad.numpy(), f"{name}_scores": scores,
                      f"{name}_n": np.int64(n)})
    # DRModel.forward end-to-end (encoder + scores + CE) on a tiny BERT
    from transformers import BertModel
    lm = BertModel(bw.bert_config(layers=1), add_pooling_layer=False)
    bw.init_model_(lm, 5)
    lm.train()
    data_args = SimpleNamespace(train_n_passages=2)
    train_args = SimpleNamespace(negatives_x_device=False)
    model = ref_bi.DRModel(lm_q=lm, lm_p=lm, tied=True, pooling="first", data_args=data_args,
                           train_args=train_args)
    qi, qm = bw.token_batch(4, 32, seed=1)
    pi, pm = bw.token_batch(8, 64, seed=2)
    outp = model(query={"input_ids": torch.from_numpy(qi), "attention_mask": torch.from_numpy(qm)},
                 passage={"input_ids": torch.from_numpy(pi), "attention_mask": torch.from_numpy(pm)})
    cases.update({"fwd_qids": qi, "fwd_qmask": qm, "fwd_pids": pi, "fwd_pmask": pm,
                  "fwd_loss": np.float32(outp.loss.item()), "fwd_scores": outp.scores.detach().numpy()})
    np.savez_compressed(os.path.join(OUT, "loss.npz"), **cases)


def gen_rerank():
    import DRT.model.linear as ref_linear
    import DRT.model.reranker as ref_rr
    from transformers import BertModel
    torch.manual_seed(0)
    lm = BertModel(bw.bert_config(layers=2), add_pooling_layer=False).eval()
    bw.init_model_(lm, 2)
    head = ref_linear.LinearHead(768, 1)
    with torch.no_grad():
        head.linear.weight.copy_(torch.from_numpy(bw.param_value(2, "rr_head.linear.weight", (1, 768))))
    out = {}
    ids, mask = bw.token_batch(6, 160, seed=33)
    for pooling in ("first", "mean"):
        m = ref_rr.RRModel(lm=lm, head=head, pooling=pooling).eval()
        with torch.no_grad():
            s = m(pos_pairs={"input_ids": torch.from_numpy(ids), "attention_mask": torch.from_numpy(mask)})
        out[f"scores_{pooling}"] = s.numpy()
    np.savez_compressed(os.path.join(OUT, "rerank.npz"), input_ids=ids, attention_mask=mask, **out)


def gen_metrics(ref_metrics):
    rng = np.random.default_rng(7)
    cases = []
    for Q, K, dens in [(16, 100, 0.05), (32, 1000, 0.002), (5, 20, 0.3), (8, 10, 0.0)]:
        hits = (rng.random((Q, K)) < dens).astype(np.int8)
        topk = [1, 5, 10, 20, 100, 1000][: 3 if K < 100 else 6]
        topk = [k for k in topk if k <= K] or [K]
        cases.append({"hits": hits.tolist(), "topk": topk, "metrics": ref_metrics.get_metrics(hits, topk)})
    with open(os.path.join(OUT, "metrics.json"), "w") as f:
        json.dump(cases, f)


def gen_merge(ref_utils):
    rng = np.random.default_rng(11)
    cases = []
    for parts, nq, per, topk in [(2, 3, 20, 10), (4, 5, 50, 25), (8, 2, 30, 100)]:
        results = []
        doc = 0
        for _ in range(parts):
            res = {}
            for q in range(nq):
                scores = rng.standard_normal(per)
                res[f"q{q}"] = {f"d{doc + j}": float(s) for j, s in enumerate(scores)}
            doc += per
            results.append(res)
        merged = ref_utils.merge_retrieval_results_by_score(results, topk=topk)
        cases.append({"results": results, "topk": topk,
                      "merged": {q: list(v.items()) for q, v in merged.items()}})
    with open(os.path.join(OUT, "merge.json"), "w") as f:
        json.dump(cases, f)


def corpus_topk_inputs(seed=31, n=20000, nq=16, d=768, lim=16):
    """Integer-valued embeddings (exact in bf16 and in every fp32 dot product), regenerated
    from this spec on the GPU box."""
    rng = np.random.default_rng(seed)
    q = rng.integers(-lim, lim + 1, size=(nq, d)).astype(np.float32)
    p = rng.integers(-lim, lim + 1, size=(n, d)).astype(np.float32)
    return q, p


def gen_corpus_topk(ref_utils, k=1000, parts=3):
    """Corpus-level top-k from the reference's own partition merge
    (merge_retrieval_results_by_score, DRT/model/utils.py:215-229): the corpus is cut into
    `parts` contiguous row partitions (as the sharded search cuts it), each partition's
    {doc: score} is q . p^T (biencoder.py:107), and the reference keeps the top k.  Python's
    sort is stable, so equal scores keep insertion (= ascending doc id) order."""
    q, p = corpus_topk_inputs()
    scores = q.astype(np.float64) @ p.astype(np.float64).T
    n = p.shape[0]
    bounds = np.linspace(0, n, parts + 1).astype(int)
    results = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        results.append({f"q{r}": {j: float(scores[r, j]) for j in range(a, b)} for r in range(q.shape[0])})
    merged = ref_utils.merge_retrieval_results_by_score(results, topk=k)
    ids = np.array([list(merged[f"q{r}"].keys()) for r in range(q.shape[0])], dtype=np.int32)
    sc = np.array([list(merged[f"q{r}"].values()) for r in range(q.shape[0])], dtype=np.float32)
    np.savez_compressed(os.path.join(OUT, "corpus_topk.npz"), seed=31, n=n, nq=q.shape[0], d=q.shape[1], lim=16,
                        k=k, parts=parts, ids=ids, scores=sc)


def answer_cases(seed=21, n_docs=60, n_queries=40):
    """Synthetic passages / answer lists for has_answers (uncased, NFD, punctuation,
    accents, multi-token answers, answers absent from every passage, empty answers)."""
    rng = np.random.default_rng(seed)
    words = ["Paris", "paris", "the", "Eiffel", "Tower", "tower", "1889", "Caf\u00e9", "cafe\u0301", "New",
             "York", "new-york", "U.S.", "u.s", "\u00c9cole", "ecole", "x", "42", "forty-two", "\u6771\u4eac",
             "na\u00efve", "ma\u00f1ana", "O'Neil", "it's", "(1)", "rock", "and", "roll", "rock'n'roll", ","]
    docs = [" ".join(rng.choice(words, size=int(rng.integers(0, 40)))) for _ in range(n_docs)]
    cases = []
    for _ in range(n_queries):
        na = int(rng.integers(0, 4))
        ans = [" ".join(rng.choice(words, size=int(rng.integers(1, 4)))) for _ in range(na)]
        if rng.random() < 0.1:
            ans.append("")
        if rng.random() < 0.2:
            ans.append("zzz not present")
        sel = rng.choice(n_docs, size=int(rng.integers(1, 25)), replace=True).tolist()
        cases.append({"answers": ans, "docs": sel})
    return docs, cases


def gen_answers():
    import DRT.evaluator.nq_eval as ref_nq
    docs, cases = answer_cases()
    for c in cases:
        c["has"] = [int(ref_nq.has_answers(docs[j], c["answers"])) for j in c["docs"]]
    with open(os.path.join(OUT, "answers.json"), "w", encoding="utf-8") as f:
        json.dump({"docs": docs, "cases": cases}, f, ensure_ascii=False)


def main():
    os.makedirs(OUT, exist_ok=True)
    ref_bi, ref_linear, ref_utils, ref_losses, ref_metrics = _ref()
    variants = [(p, n, h) for p in ("first", "mean", "max") for n in (False, True) for h in (False, True)]
    gen_encode(ref_bi, ref_linear, layers=2, seed=0, variants=variants, B=8, L=64, tag="l2")
    gen_encode(ref_bi, ref_linear, layers=12, seed=1, variants=[("first", False, False), ("mean", True, False)],
               B=4, L=128, tag="l12")
    gen_loss(ref_bi, ref_losses)
    gen_metrics(ref_metrics)
    gen_merge(ref_utils)
    gen_corpus_topk(ref_utils)
    gen_rerank()
    gen_answers()
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
