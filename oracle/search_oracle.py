"""CPU restatement of the reference's brute-force search — TEST INFRASTRUCTURE ONLY.

Restates, in numpy:

* ``BaseFaissIPRetriever.search`` (DRT/evaluator/index.py:31-33): exact
  inner-product k-NN (``faiss.IndexFlatIP(d)``, index.py:19/23), results in
  descending score order.  faiss is a third-party dependency that is NOT
  installed in this image and that the reference does not pin (no
  requirements file); the restated semantics are faiss's published ones for
  IndexFlatIP: exact fp32 dot products, top-k by descending score, rows past
  ``ntotal`` padded with label -1 and ``numeric_limits<float>::lowest()``.
  The reference re-sorts with ``np.argsort(-scores)`` (default quicksort:
  tie order unspecified); the oracle pins ties to ascending id — a
  deterministic refinement of the reference order, which the GPU path
  follows bit for bit.
* the partition merge that replaces the reference's shard exchange
  (trainer.py:220-262 concatenates per-rank shards into one index;
  DRT/model/utils.py:215-229 ``merge_retrieval_results_by_score`` keeps the
  top-k by descending score over partitions).

Pinning: the score definition (q . p over the same vectors) is pinned by the
golden vectors of ``DRModel.forward`` generated from the reference
(tests/golden/), and the merge order by golden vectors of
``merge_retrieval_results_by_score``; the faiss kernel itself cannot run
here (absent), so top-k over a corpus is checked against this restatement.

Scores are accumulated in float64 (exact for the bf16-valued inputs the
tests use when |values| are small integers; within 1e-7 relative otherwise)
and reported as float32.
"""
from __future__ import annotations

import numpy as np

PAD_SCORE = np.float32(np.finfo(np.float32).min)  # faiss CMin<float>::neutral()
PAD_ID = -1


# ---------------------------------------------------------------------------
# bf16 helpers (round-to-nearest-even, as torch's .to(torch.bfloat16))
# ---------------------------------------------------------------------------
def bf16_bits(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    rounded = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    nan = np.isnan(x)
    out = rounded.astype(np.uint16)
    if nan.any():
        out[nan] = 0x7FC0
    return out


def bf16_from_bits(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def bf16_round(x: np.ndarray) -> np.ndarray:
    """fp32 -> nearest bf16 value, returned as fp32."""
    return bf16_from_bits(bf16_bits(x))


# ---------------------------------------------------------------------------
# exact top-k with the (score desc, id asc) total order
# ---------------------------------------------------------------------------
def _order(scores: np.ndarray, ids: np.ndarray) -> np.ndarray:
    # lexsort: last key is primary -> primary = -score (desc), secondary = id asc
    return np.lexsort((ids, -scores))


def ip_topk(q: np.ndarray, p: np.ndarray, k: int, id_offset: int = 0, chunk: int = 262144,
            dtype=np.float64):
    """Exact IP top-k of q [nq, d] over p [n, d].  Returns (scores f32 [nq,k], ids i64 [nq,k])."""
    q = np.asarray(q)
    p = np.asarray(p)
    nq = q.shape[0]
    n = p.shape[0]
    out_s = np.full((nq, k), PAD_SCORE, dtype=np.float32)
    out_i = np.full((nq, k), PAD_ID, dtype=np.int64)
    if nq == 0 or n == 0:
        return out_s, out_i
    qd = q.astype(dtype, copy=False)
    best_s = np.empty((nq, 0), dtype=dtype)
    best_i = np.empty((nq, 0), dtype=np.int64)
    for c0 in range(0, n, chunk):
        pc = p[c0:c0 + chunk].astype(dtype, copy=False)
        s = qd @ pc.T                                     # [nq, c]
        ids = np.arange(c0, c0 + pc.shape[0], dtype=np.int64)
        if s.shape[1] > k:
            # keep a superset: everything >= the k-th largest value (ties kept)
            kth = np.partition(s, s.shape[1] - k, axis=1)[:, s.shape[1] - k][:, None]
            keep = s >= kth
            cs = [s[r][keep[r]] for r in range(nq)]
            ci = [ids[keep[r]] for r in range(nq)]
        else:
            cs = [s[r] for r in range(nq)]
            ci = [ids for _ in range(nq)]
        new_s, new_i = [], []
        for r in range(nq):
            ss = np.concatenate([best_s[r], cs[r]])
            ii = np.concatenate([best_i[r], ci[r]])
            o = _order(ss, ii)[:k]
            new_s.append(ss[o])
            new_i.append(ii[o])
        w = max(len(x) for x in new_s)
        best_s = np.full((nq, w), -np.inf, dtype=dtype)
        best_i = np.full((nq, w), np.iinfo(np.int64).max, dtype=np.int64)
        for r in range(nq):
            best_s[r, :len(new_s[r])] = new_s[r]
            best_i[r, :len(new_i[r])] = new_i[r]
    kk = min(k, n)
    out_s[:, :kk] = best_s[:, :kk].astype(np.float32)
    out_i[:, :kk] = best_i[:, :kk] + id_offset
    return out_s, out_i


def search_ids(q: np.ndarray, p: np.ndarray, k: int) -> np.ndarray:
    """What BaseFaissIPRetriever.search returns (index.py:31-33): ids only, [nq, k] int64."""
    return ip_topk(q, p, k)[1]


def merge_topk(scores: np.ndarray, ids: np.ndarray, k_out: int):
    """Merge per-part sorted lists [nparts, nq, k_in] into the top-k_out (score desc, id asc)."""
    nparts, nq, k_in = scores.shape
    out_s = np.full((nq, k_out), PAD_SCORE, dtype=np.float32)
    out_i = np.full((nq, k_out), PAD_ID, dtype=np.int64)
    for r in range(nq):
        ss = scores[:, r, :].reshape(-1).astype(np.float32)
        ii = ids[:, r, :].reshape(-1).astype(np.int64)
        o = _order(ss.astype(np.float64), ii)[:k_out]
        out_s[r, :len(o)] = ss[o]
        out_i[r, :len(o)] = ii[o]
    return out_s, out_i


def shard_bounds(n: int, world: int, rank: int):
    """Contiguous row shard of rank r: [r*ceil(n/W), min(n, (r+1)*ceil(n/W)))."""
    per = -(-n // world) if world > 0 else n
    lo = min(n, rank * per)
    hi = min(n, lo + per)
    return lo, hi
