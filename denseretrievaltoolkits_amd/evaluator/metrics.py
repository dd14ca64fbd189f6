"""Recall / MRR / NDCG over a binary hit matrix — same semantics as
DRT/evaluator/metrics.py:4-59 (a CPU consumer of the search output, kept so
Trainer.evaluate reports identical numbers):

* recall@k: number of rows whose FIRST hit is at position < k (a sum, not a mean);
* mrr@k:    sum over rows of 1/(pos+1) of the first hit if pos < k;
* ndcg@k:   batch-level ratio sum(DCG@k) / sum(IDCG@k) with natural-log
            discounts, IDCG over max(#hits in the row, 1) ideal positions.
"""
from __future__ import annotations

import math
from typing import Dict, Sequence

import numpy as np


def _first_hit(hits: np.ndarray) -> np.ndarray:
    any_hit = hits.any(axis=1)
    first = np.where(any_hit, hits.argmax(axis=1), np.iinfo(np.int64).max)
    return first


def recall(indices, topk: Sequence[int]):
    hits = np.asarray(indices) != 0
    first = _first_hit(hits)
    return [int((first < k).sum()) for k in topk]


def mrr(indices, topk: Sequence[int]):
    hits = np.asarray(indices) != 0
    first = _first_hit(hits)
    out = []
    for k in topk:
        sel = first < k
        out.append(float(np.sum(1.0 / (first[sel] + 1))) if sel.any() else 0)
    return out


def ndcg(indices, topk: Sequence[int]):
    hits = np.asarray(indices) != 0
    nrow, ncol = hits.shape if hits.ndim == 2 else (0, 0)
    disc = 1.0 / np.log(np.arange(max(ncol, 1)) + 2.0)
    out = []
    cnt = hits.sum(axis=1) if nrow else np.zeros(0, dtype=np.int64)
    for k in topk:
        dcg = float((hits[:, :k] * disc[:k]).sum()) if nrow else 0.0
        idcg = 0.0
        for c in np.maximum(cnt, 1):
            idcg += float(disc[: min(int(c), k)].sum()) if k > 0 else 0.0
        out.append(dcg / idcg if idcg else math.nan)
    return out


def get_metrics(indices, topk: Sequence[int]) -> Dict[str, float]:
    r, m, n = recall(indices, topk), mrr(indices, topk), ndcg(indices, topk)
    res = {}
    for name, vals in zip(["Recall@", "MRR@", "NDCG@"], [r, m, n]):
        for k, v in zip(topk, vals):
            res[name + str(k)] = v
    return res
