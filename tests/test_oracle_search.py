"""CPU: the search oracle against naive brute force and the reference's merge semantics."""
import numpy as np
import pytest

from helpers import int_bf16
from oracle import search_oracle as orc


def naive_topk(q, p, k):
    s = q.astype(np.float64) @ p.astype(np.float64).T
    out_s = np.full((q.shape[0], k), orc.PAD_SCORE, np.float32)
    out_i = np.full((q.shape[0], k), -1, np.int64)
    for r in range(q.shape[0]):
        order = sorted(range(p.shape[0]), key=lambda j: (-s[r, j], j))[:k]
        out_s[r, :len(order)] = s[r, order]
        out_i[r, :len(order)] = order
    return out_s, out_i


@pytest.mark.parametrize("n,k,chunk", [(300, 10, 64), (50, 100, 16), (257, 257, 1000), (1000, 1, 7)])
def test_oracle_matches_naive(n, k, chunk):
    rng = np.random.default_rng(n + k)
    q = int_bf16(rng, (4, 16), -2, 2)     # lots of exact ties
    p = int_bf16(rng, (n, 16), -2, 2)
    s, i = orc.ip_topk(q, p, k, chunk=chunk)
    es, ei = naive_topk(q, p, k)
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(s, es)


def test_oracle_id_offset_and_empty():
    rng = np.random.default_rng(0)
    q = int_bf16(rng, (2, 8))
    s, i = orc.ip_topk(q, np.zeros((0, 8), np.float32), 5)
    assert (i == -1).all() and (s == orc.PAD_SCORE).all()
    p = int_bf16(rng, (20, 8))
    s0, i0 = orc.ip_topk(q, p, 5)
    s1, i1 = orc.ip_topk(q, p, 5, id_offset=100)
    np.testing.assert_array_equal(i1, i0 + 100)


def test_merge_of_shards_equals_whole():
    rng = np.random.default_rng(1)
    q = int_bf16(rng, (3, 32))
    p = int_bf16(rng, (1001, 32))
    whole = orc.ip_topk(q, p, 50)
    parts = [orc.ip_topk(q, p[lo:hi], 50, id_offset=lo) for lo, hi in
             (orc.shard_bounds(1001, 4, r) for r in range(4))]
    ms, mi = orc.merge_topk(np.stack([a for a, _ in parts]), np.stack([b for _, b in parts]), 50)
    np.testing.assert_array_equal(mi, whole[1])
    np.testing.assert_array_equal(ms, whole[0])


def test_shard_bounds_cover_rows_once():
    for n in (0, 1, 7, 10_000_000):
        for w in (1, 2, 3, 8):
            spans = [orc.shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, _) in zip(spans, spans[1:]):
                assert b == c and a <= b


def test_bf16_round_matches_torch():
    import torch
    x = np.random.default_rng(2).standard_normal(10000).astype(np.float32) * 100
    ref = torch.from_numpy(x).to(torch.bfloat16).float().numpy()
    np.testing.assert_array_equal(orc.bf16_round(x), ref)


# ---------------------------------------------------------------------------
# global-threshold protocol restatement == single-index oracle
# ---------------------------------------------------------------------------
def _protocol(q, p, k, world):
    n = p.shape[0]
    bounds = [orc.shard_bounds(n, world, r) for r in range(world)]
    lists = np.stack([orc.dist_sample(q, p[lo:hi], n, k) for lo, hi in bounds])
    tau = orc.dist_tau(lists, k)
    parts = np.stack([orc.dist_filter(q, p[lo:hi], n, k, lo, tau) for lo, hi in bounds])
    return orc.merge_packed(parts, k, n), tau


@pytest.mark.parametrize("world,n,k", [(2, 40000, 20), (3, 17000, 50), (4, 1000, 30), (2, 10, 30)])
def test_global_tau_protocol_matches_single_index(world, n, k):
    rng = np.random.default_rng(n + k)
    p = rng.integers(-8, 9, size=(n, 16)).astype(np.float32)
    q = rng.integers(-8, 9, size=(4, 16)).astype(np.float32)
    (s, i, st), tau = _protocol(q, p, k, world)
    es, ei = orc.ip_topk(q, p, k)
    assert (st == 0).all()
    assert np.array_equal(i, ei) and np.array_equal(s, es)
    if n <= 4 * max(4096, 4 * k):
        assert np.isneginf(tau).all()


def test_global_tau_protocol_flags_too_high_threshold():
    rng = np.random.default_rng(3)
    p = rng.integers(-8, 9, size=(40000, 16)).astype(np.float32)
    q = rng.integers(-8, 9, size=(2, 16)).astype(np.float32)
    k = 20
    n = p.shape[0]
    tau = np.full(2, 1e9, np.float32)          # nothing passes: fewer than k candidates
    parts = np.stack([orc.dist_filter(q, p[lo:hi], n, k, lo, tau)
                      for lo, hi in (orc.shard_bounds(n, 2, r) for r in range(2))])
    _, _, st = orc.merge_packed(parts, k, n)
    assert (st == 1).all()


def test_desc_key_roundtrip_and_order():
    x = np.array([3.5, -0.0, 0.0, -2.25, np.float32(np.finfo(np.float32).min), 1e30], np.float32)
    k = orc.desc_key(x)
    assert np.array_equal(orc.desc_key_to_score(k), x + np.float32(0.0))
    assert np.array_equal(np.argsort(k, kind="stable"), np.argsort(-(x + 0.0), kind="stable"))
