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
            dtype=np.float64, out_dtype=np.float32):
    """Exact IP top-k of q [nq, d] over p [n, d].  Returns (scores [nq,k] in out_dtype (fp32: the
    faiss output type; fp64 keeps the ranking precision for a later partition merge), ids i64)."""
    q = np.asarray(q)
    p = np.asarray(p)
    nq = q.shape[0]
    n = p.shape[0]
    out_s = np.full((nq, k), PAD_SCORE, dtype=out_dtype)
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
    out_s[:, :kk] = best_s[:, :kk].astype(out_dtype)
    out_i[:, :kk] = best_i[:, :kk] + id_offset
    return out_s, out_i


def search_ids(q: np.ndarray, p: np.ndarray, k: int) -> np.ndarray:
    """What BaseFaissIPRetriever.search returns (index.py:31-33): ids only, [nq, k] int64."""
    return ip_topk(q, p, k)[1]


def merge_topk(scores: np.ndarray, ids: np.ndarray, k_out: int):
    """Merge per-part sorted lists [nparts, nq, k_in] into the top-k_out (score desc, id asc).
    fp64 scores are merged (and returned) in fp64, anything else in fp32."""
    nparts, nq, k_in = scores.shape
    sdt = np.float64 if scores.dtype == np.float64 else np.float32
    out_s = np.full((nq, k_out), PAD_SCORE, dtype=sdt)
    out_i = np.full((nq, k_out), PAD_ID, dtype=np.int64)
    for r in range(nq):
        ss = scores[:, r, :].reshape(-1).astype(sdt)
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


# ---------------------------------------------------------------------------
# Global-threshold distributed protocol (csrc/search.hip drt_ip_topk_dist_*).
# Not a reference algorithm: the reference concatenates shards into ONE faiss
# index (trainer.py:220-262); the protocol must reproduce exactly that
# single-index result, which is what the tests check, so this restatement
# only has to agree with the GPU kernels on the exchanged intermediate data.
# ---------------------------------------------------------------------------
PAD_KEY32 = np.uint32(0xFFFFFFFF)
PAD_KEY64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def desc_key(scores: np.ndarray) -> np.ndarray:
    """uint32 whose ascending order is descending score (drt_common.h desc_key)."""
    s = np.asarray(scores, dtype=np.float32) + np.float32(0.0)
    u = s.view(np.uint32)
    ordk = np.where(u & np.uint32(0x80000000), ~u, u | np.uint32(0x80000000)).astype(np.uint32)
    return (~ordk).astype(np.uint32)


def desc_key_to_score(k: np.ndarray) -> np.ndarray:
    ordk = ~np.asarray(k, dtype=np.uint32)
    u = np.where(ordk & np.uint32(0x80000000), ordk & np.uint32(0x7FFFFFFF), ~ordk).astype(np.uint32)
    return u.view(np.float32)


def _poisson_tail_ge(lam, r):
    import math
    p = math.exp(-lam + r * math.log(lam) - math.lgamma(r + 1.0))
    s = 0.0
    i = r
    while i < r + 2000:
        s += p
        p *= lam / (i + 1)
        i += 1
        if p < 1e-30 * s:
            break
    return s


def sample_rank(k: int) -> int:
    """drt_ip_topk_sample_rank: smallest r with P[Poisson(k r / target) >= r] < 1e-9."""
    target = max(4096, 4 * k)
    r = 1
    while _poisson_tail_ge(k * r / target, r) > 1e-9 and r < 100000:
        r += 1
    return r


def dist_plan(n_local: int, n_global: int, k: int):
    """make_dist_plan: (sample?, r, sampled row indices of this shard, cap)."""
    target = max(4096, 4 * k)
    cap = 4 * target
    sample = n_global > cap
    r = sample_rank(k) if sample else 0
    rows = np.zeros(0, np.int64)
    if sample and n_local > 0:
        m = min(n_local, (r * n_local + target - 1) // target)
        m_cap = max(1, 4096 // r) * 4096
        m = min(m, m_cap)
        stride = max(1, n_local // m)
        m = min((n_local - stride // 2 + stride - 1) // stride, m_cap)
        rows = np.arange(m, dtype=np.int64) * stride + stride // 2
    return dict(sample=sample, r=sample_rank(k), rows=rows, cap=cap, target=target)


def _scores_f32(q, p):
    return (np.asarray(q, np.float64) @ np.asarray(p, np.float64).T).astype(np.float32)


def dist_sample(q, p_local, n_global, k):
    """Best r sampled desc-keys per query, ascending, padded with 0xFFFFFFFF -> uint32 [nq, r]."""
    plan = dist_plan(p_local.shape[0], n_global, k)
    r = plan["r"]
    nq = np.asarray(q).shape[0]
    out = np.full((nq, r), PAD_KEY32, dtype=np.uint32)
    if not plan["sample"] or len(plan["rows"]) == 0:
        return out
    keys = np.sort(desc_key(_scores_f32(q, p_local[plan["rows"]])), axis=1)[:, :r]
    out[:, :keys.shape[1]] = keys
    return out


def dist_tau(lists, k):
    """tau[q] = score of the r-th smallest key over [nlists, nq, r] (-inf if fewer than r real keys)."""
    lists = np.asarray(lists, dtype=np.uint32)
    r = sample_rank(k)
    allk = np.sort(np.transpose(lists, (1, 0, 2)).reshape(lists.shape[1], -1), axis=1)
    kr = allk[:, r - 1]
    tau = desc_key_to_score(kr).copy()
    tau[kr == PAD_KEY32] = -np.inf
    return tau.astype(np.float32)


def dist_filter(q, p_local, n_global, k, id_offset, tau):
    """Packed uint64 [nq, k + 1]: sorted (desc_key << 32 | global id) of rows with score >= tau;
    entry k = (valid entries << 32) | flags (bit 0: more than cap candidates, i.e. the GPU buffer
    overflowed)."""
    plan = dist_plan(p_local.shape[0], n_global, k)
    nq = np.asarray(q).shape[0]
    out = np.full((nq, k + 1), PAD_KEY64, dtype=np.uint64)
    out[:, k] = 0
    if p_local.shape[0] == 0:
        return out
    s = _scores_f32(q, p_local)
    for i in range(nq):
        sel = np.nonzero(s[i] >= tau[i])[0]
        if len(sel) > plan["cap"]:
            out[i, k] = 1
        if len(sel) > k:   # truncated: more hits than the list carries (bit 1, round 6)
            out[i, k] |= np.uint64(2)
        keys = (desc_key(s[i, sel]).astype(np.uint64) << np.uint64(32)) | (sel + id_offset).astype(np.uint64)
        keys = np.sort(keys)[:k]
        out[i, :len(keys)] = keys
        out[i, k] |= np.uint64(len(keys)) << np.uint64(32)
    return out


def merge_packed(parts, k, n_global, k_cert=None):
    """[nparts, nq, lcap + 1] packed lists (lcap <= k) -> (scores f32 [nq,k], ids i64 [nq,k], status i32
    [nq]).  Capped lists (lcap < k, round 6): a list flagged truncated (bit 1) whose last entry ranks above
    the k-th merged place leaves its query uncertified."""
    parts = np.asarray(parts, dtype=np.uint64)
    nparts, nq, w = parts.shape
    lcap = w - 1
    kc = k if k_cert is None else k_cert
    allk = np.sort(np.transpose(parts[:, :, :lcap], (1, 0, 2)).reshape(nq, -1), axis=1)
    keys = np.full((nq, k), PAD_KEY64, dtype=np.uint64)
    keys[:, :min(k, allk.shape[1])] = allk[:, :k]
    pad = keys == PAD_KEY64
    s = desc_key_to_score((keys >> np.uint64(32)).astype(np.uint32)).copy()
    ids = (keys & np.uint64(0xFFFFFFFF)).astype(np.int64)
    s[pad] = PAD_SCORE
    ids[pad] = PAD_ID
    over = (parts[:, :, lcap] & np.uint64(1)).any(axis=0)
    bad = over | (pad[:, kc - 1] & (n_global >= kc))
    if lcap < k:
        for qi in range(nq):
            for l in range(nparts):
                lst = parts[l, qi, :lcap]
                cnt = int((lst != PAD_KEY64).sum())
                if (parts[l, qi, lcap] & np.uint64(2)) and cnt == lcap:
                    rank = int(np.searchsorted(allk[qi], lst[cnt - 1]))   # keys are unique
                    if rank < k - 1:
                        bad[qi] = True
    return s.astype(np.float32), ids, bad.astype(np.int32)


# ---------------------------------------------------------------------------
# Sharded search at k > 2048 (csrc/search.hip drt_ip_topk_large_keys + drt_merge_exact, round 6): every
# shard's canonical top-k carries each entry's EXACT order key; the lists are merged by (key, global id).
# Like the protocol above this only restates the exchanged data; the tests check the end result against
# the single-index ip_topk.
# ---------------------------------------------------------------------------
def desc_key64(scores: np.ndarray) -> np.ndarray:
    """uint64 whose ascending order is descending fp64 score (search.hip desc_key64)."""
    s = np.asarray(scores, dtype=np.float64) + 0.0
    u = s.view(np.uint64)
    neg = (u >> np.uint64(63)) != 0
    ordk = np.where(neg, ~u, u | np.uint64(0x8000000000000000))
    return ~ordk


def exact_keys_topk(q, p_local, k, id_offset=0):
    """(keys uint64 [nq, k], ids int64 [nq, k]) of a shard's canonical top-k; (~0, -1) pads."""
    s, i = ip_topk(q, p_local, k, id_offset=id_offset, dtype=np.float64, out_dtype=np.float64)
    keys = desc_key64(s)
    keys[i < 0] = PAD_KEY64
    return keys, i


def merge_exact(keys, ids, k):
    """Top-k of [nparts, nq, k] (key, id) lists by (key asc, id asc) -> (scores fp32, ids)."""
    nparts, nq, _ = keys.shape
    out_s = np.full((nq, k), PAD_SCORE, dtype=np.float32)
    out_i = np.full((nq, k), PAD_ID, dtype=np.int64)
    for r in range(nq):
        kk = keys[:, r, :].reshape(-1)
        ii = ids[:, r, :].reshape(-1)
        real = kk != PAD_KEY64
        kk, ii = kk[real], ii[real]
        o = np.lexsort((ii, kk))[:k]
        ordk = ~kk[o]
        u = np.where((ordk >> np.uint64(63)) != 0, ordk & np.uint64(0x7FFFFFFFFFFFFFFF), ~ordk)
        out_s[r, :len(o)] = u.view(np.float64).astype(np.float32)
        out_i[r, :len(o)] = ii[o]
    return out_s, out_i
