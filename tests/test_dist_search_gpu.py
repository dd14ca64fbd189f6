"""GPU parity of the global-threshold distributed protocol (drt_ip_topk_dist_*,
drt_topk_merge_packed), shards simulated on one GPU.

Reference behaviour: the reference concatenates every rank's shard into one
faiss IndexFlatIP (DRT/trainer/trainer.py:220-262) and searches it
(DRT/evaluator/index.py:31-33); the protocol must return exactly that
single-index top-k.  Integer-valued inputs make every score exact, so the
exchanged intermediates (sample keys, tau, packed lists) are compared with the
oracle restatement bit for bit as well as the final (scores, ids).
"""
import numpy as np
import pytest

from helpers import int_bf16, gauss_bf16, to_dev_bf16
from oracle import search_oracle as orc

pytestmark = pytest.mark.gpu


def _gpu_protocol(dev, q, p, k, world, check_intermediates=True):
    import torch
    from denseretrievaltoolkits_amd import kernels
    n = p.shape[0]
    d = q.shape[1]
    qt = to_dev_bf16(q, dev)
    bounds = [orc.shard_bounds(n, world, r) for r in range(world)]
    shards = [to_dev_bf16(p[lo:hi], dev) if hi > lo else torch.empty((0, d), dtype=torch.bfloat16, device=dev)
              for lo, hi in bounds]
    lists = torch.stack([kernels.dist_sample(qt, sh, n, k) for sh in shards])
    tau = kernels.dist_tau(lists, k)
    parts = torch.stack([kernels.dist_filter(qt, sh, n, k, lo, tau) for sh, (lo, _) in zip(shards, bounds)])
    # the fused tau + filter entry (the path ShardedFlatIP takes) gives the same packed lists
    fused = torch.stack([kernels.dist_filter_lists(qt, sh, n, k, lo, lists) for sh, (lo, _) in zip(shards, bounds)])
    assert torch.equal(fused, parts)
    s, i, st = kernels.merge_packed(parts, k, n)
    torch.cuda.synchronize()
    if check_intermediates:
        e_lists = np.stack([orc.dist_sample(q, p[lo:hi], n, k) for lo, hi in bounds])
        np.testing.assert_array_equal(lists.cpu().numpy().view(np.uint32), e_lists)
        e_tau = orc.dist_tau(e_lists, k)
        np.testing.assert_array_equal(tau.cpu().numpy(), e_tau)
        e_parts = np.stack([orc.dist_filter(q, p[lo:hi], n, k, lo, e_tau) for lo, hi in bounds])
        np.testing.assert_array_equal(parts.cpu().numpy().view(np.uint64), e_parts)
    return s.cpu().numpy(), i.cpu().numpy(), st.cpu().numpy()


@pytest.mark.parametrize("world,nq,n,d,k", [
    (8, 128, 400000, 768, 1000),   # N=8 shape of the bench (sampled global tau)
    (2, 16, 50000, 768, 1000),
    (3, 33, 100003, 128, 100),     # ragged shards
    (4, 5, 12000, 64, 10),         # n_global <= cap: tau = -inf, everything filtered
    (5, 4, 3, 128, 10),            # fewer rows than k, empty shards
    (2, 7, 60000, 1024, 2048),     # k at its maximum
    # more than 128 queries in one launch: the 32-queries-per-wave filter kernel (ip_scan32r), full
    # and partial 256-query blocks, ragged shards (partial 16-row tiles), several d
    (2, 300, 30000, 768, 1000),
    (3, 129, 20011, 320, 100),
    (1, 257, 5003, 64, 10),
    (2, 520, 40000, 576, 200),
])
def test_dist_protocol_integer_bit_exact(dev, world, nq, n, d, k):
    rng = np.random.default_rng(world * 7 + n + d + k)
    q = int_bf16(rng, (nq, d), -4, 4)
    p = int_bf16(rng, (n, d), -4, 4)
    s, i, st = _gpu_protocol(dev, q, p, k, world)
    es, ei = orc.ip_topk(q, p, k)
    assert (st == 0).all()
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(s, es)


def test_dist_protocol_gaussian(dev):
    rng = np.random.default_rng(11)
    world, nq, n, d, k = 8, 64, 240000, 768, 1000
    q = gauss_bf16(rng, (nq, d))
    p = gauss_bf16(rng, (n, d))
    s, i, st = _gpu_protocol(dev, q, p, k, world, check_intermediates=False)
    assert (st == 0).all()
    es, ei = orc.ip_topk(q, p, k)
    np.testing.assert_allclose(s, es, atol=1e-3, rtol=0)
    assert (i == ei).mean() > 0.999


def test_dist_protocol_equals_single_gpu_search(dev):
    """Gaussian data: global-tau result == single-index HIP result bit for bit (same kernels' fp32 scores)."""
    import torch
    from denseretrievaltoolkits_amd import kernels
    rng = np.random.default_rng(12)
    world, nq, n, d, k = 4, 32, 200000, 768, 1000
    q = gauss_bf16(rng, (nq, d))
    p = gauss_bf16(rng, (n, d))
    s, i, st = _gpu_protocol(dev, q, p, k, world, check_intermediates=False)
    s1, i1, _ = kernels.ip_topk(to_dev_bf16(q, dev), to_dev_bf16(p, dev), k)
    assert (st == 0).all()
    np.testing.assert_array_equal(i, i1.cpu().numpy())
    np.testing.assert_array_equal(s, s1.cpu().numpy())


def test_dist_overflow_and_short_lists_are_flagged(dev):
    import torch
    from denseretrievaltoolkits_amd import kernels
    rng = np.random.default_rng(5)
    nq, n, d, k = 3, 80000, 128, 50
    q = int_bf16(rng, (nq, d), -4, 4)
    p = int_bf16(rng, (n, d), -4, 4)
    qt, pt = to_dev_bf16(q, dev), to_dev_bf16(p, dev)
    # tau = -inf on a shard bigger than cap: overflow flag, status 1
    tau = torch.full((nq,), float("-inf"), device=dev)
    parts = kernels.dist_filter(qt, pt, n, k, 0, tau)[None]
    assert (parts[0, :, k].cpu().numpy() & 1).all()
    _, _, st = kernels.merge_packed(parts, k, n)
    assert (st.cpu().numpy() == 1).all()
    # tau above every score: no candidates, status 1
    tau = torch.full((nq,), 1e9, device=dev)
    parts = kernels.dist_filter(qt, pt, n, k, 0, tau)[None]
    s, i, st = kernels.merge_packed(parts, k, n)
    assert (st.cpu().numpy() == 1).all()
    assert (i.cpu().numpy() == -1).all()


def test_dist_shape_errors(dev):
    import torch
    from denseretrievaltoolkits_amd import _native, kernels
    qt = torch.zeros((2, 128), dtype=torch.bfloat16, device=dev)
    pt = torch.zeros((10, 128), dtype=torch.bfloat16, device=dev)
    tau = torch.zeros((2,), device=dev)
    with pytest.raises(ValueError):
        kernels.dist_filter(qt, pt, 5, 10, 0, tau)                 # n_global < n_local
    with pytest.raises(ValueError):
        kernels.dist_filter(qt, pt, 12, 10, 5, tau)                # id_offset + n_local > n_global
    with pytest.raises(ValueError):
        kernels.dist_tau(torch.zeros((400, 2, kernels.sample_rank(1000)), dtype=torch.int32, device=dev), 1000)
    assert kernels.sample_rank(1000) == orc.sample_rank(1000)


@pytest.mark.parametrize("nparts,nq,k,fill", [(8, 128, 1000, 0.5), (2, 5, 2048, 1.0), (3, 7, 100, 0.0),
                                              (5, 9, 10, 0.3), (9, 4, 1000, 0.4), (16, 3, 1000, 0.2),
                                              (8, 2, 1000, 0.05), (1, 6, 64, 0.7), (5, 3, 2048, 0.6),
                                              (8, 3, 2048, 1.0), (6, 4, 1500, 0.95)])
@pytest.mark.parametrize("count_word", [True, False])
def test_merge_packed_vs_oracle(dev, nparts, nq, k, fill, count_word):
    """drt_topk_merge_packed against the oracle on random packed lists (unique keys, ragged fills,
    empty parts, overflow flags) for every kernel the shape selects: count merge (2-8 parts,
    nparts * k <= 16384, incl. full lists at that bound), tree merge (more parts or keys), plain
    per-query merge (one part).
    count_word False: entry k carries the flags only (the pre-0.3 contract) -> the count merge
    measures each list itself and must give the same result."""
    import torch
    from denseretrievaltoolkits_amd import kernels
    rng = np.random.default_rng(nparts * 1000 + k)
    parts = np.full((nparts, nq, k + 1), np.iinfo(np.uint64).max, dtype=np.uint64)
    n_global = nparts * k * 4
    for q in range(nq):
        ids = rng.permutation(n_global)[: nparts * k].astype(np.uint64)
        sc = rng.integers(0, 1 << 20, size=nparts * k).astype(np.uint64)   # ties across parts, ids break them
        keys = (sc << np.uint64(32)) | ids
        for l in range(nparts):
            cnt = int(rng.binomial(k, fill)) if fill < 1.0 else k
            parts[l, q, :cnt] = np.sort(keys[l * k: l * k + cnt])
            cw = np.uint64(cnt) << np.uint64(32) if count_word else np.uint64(0)
            parts[l, q, k] = cw | np.uint64(rng.random() < 0.1)  # count | overflow
    es, ei, est = orc.merge_packed(parts, k, n_global)
    pt = torch.from_numpy(parts.view(np.int64)).to(dev)
    s, i, st = kernels.merge_packed(pt, k, n_global)
    np.testing.assert_array_equal(i.cpu().numpy(), ei)
    np.testing.assert_array_equal(s.cpu().numpy(), es)
    np.testing.assert_array_equal(st.cpu().numpy(), est)


@pytest.mark.parametrize("nparts,lcap,k,fill", [(8, 256, 1256, 0.15), (4, 448, 1256, 0.3), (2, 832, 1256, 0.7),
                                                 (3, 96, 200, 0.4)])
def test_merge_packed_capped_vs_oracle(dev, nparts, lcap, k, fill):
    """Capped exchange lists (round 6): each part carries its best lcap < k keys; a part flagged truncated
    (bit 1) whose last key ranks above the k-th merged place must leave its query uncertified -- GPU ==
    oracle on random lists built to hit both sides of that rule."""
    import torch
    from denseretrievaltoolkits_amd import kernels
    rng = np.random.default_rng(nparts * 7 + lcap)
    nq = 64
    n_global = nparts * k * 4
    parts = np.full((nparts, nq, lcap + 1), np.iinfo(np.uint64).max, dtype=np.uint64)
    for q in range(nq):
        ids = rng.permutation(n_global)[: nparts * lcap].astype(np.uint64)
        # some queries skew one part's scores upward (its truncated tail reaches into the top k)
        skew = rng.random() < 0.3
        sc = rng.integers(0, 1 << 20, size=nparts * lcap).astype(np.uint64)
        for l in range(nparts):
            cnt = lcap if rng.random() < 0.5 else int(rng.binomial(lcap, fill))
            ks = sc[l * lcap: l * lcap + cnt] // (np.uint64(8) if (skew and l == 0) else np.uint64(1))
            keys = np.sort((ks << np.uint64(32)) | ids[l * lcap: l * lcap + cnt])
            parts[l, q, :cnt] = keys
            trunc = cnt == lcap and rng.random() < 0.8
            parts[l, q, lcap] = (np.uint64(cnt) << np.uint64(32)) | (np.uint64(2) if trunc else np.uint64(0))
    es, ei, est = orc.merge_packed(parts, k, n_global)
    s, i, st = kernels.merge_packed(torch.from_numpy(parts.view(np.int64)).to(dev), k, n_global)
    np.testing.assert_array_equal(i.cpu().numpy(), ei)
    np.testing.assert_array_equal(s.cpu().numpy(), es)
    np.testing.assert_array_equal(st.cpu().numpy(), est)
    assert 0 < est.sum() < nq   # both outcomes exercised


@pytest.mark.parametrize("nq,n,d,k,starts", [
    (300, 50011, 768, 1000, [0, 12000, 12000, 30001, 50011]),   # 32-query kernel, an empty chunk, ragged
    (128, 40000, 768, 100, [0, 16, 20000, 40000]),               # 16-query kernel, a one-tile chunk
    (513, 30000, 128, 200, [0, 7, 29993, 30000]),                # partial tiles at both chunk edges
    (64, 5000, 768, 10, [0, 5000]),                              # one chunk
])
def test_dist_filter_chunks_equals_whole_shard(dev, nq, n, d, k, starts):
    """kernels.dist_filter_chunks_into (one scan launch per chunk, one hit list, one select -- the grouped
    search's chunked filter) returns the packed lists of dist_filter_into over the whole shard, bit for
    bit, on integer data (exact scores) and on Gaussian data (same fp32 chains)."""
    import torch
    from denseretrievaltoolkits_amd import kernels
    rng = np.random.default_rng(nq + n + d)
    for data in ("int", "gauss"):
        if data == "int":
            q = int_bf16(rng, (nq, d), -4, 4)
            p = int_bf16(rng, (n, d), -4, 4)
        else:
            q = gauss_bf16(rng, (nq, d))
            p = gauss_bf16(rng, (n, d))
        qt, pt = to_dev_bf16(q, dev), to_dev_bf16(p, dev)
        n_global = 8 * n   # a shard of a larger corpus: sampled threshold, id offset
        off = 3 * n
        lists = kernels.dist_sample(qt, pt, n_global, k).unsqueeze(0)
        tau = kernels.dist_tau(lists, k)
        whole = torch.empty((nq, k + 1), dtype=torch.int64, device=dev)
        kernels.dist_filter_into(qt, pt, n_global, k, off, tau, whole)
        chunked = torch.full((nq, k + 1), -7, dtype=torch.int64, device=dev)
        kernels.dist_filter_chunks_into(qt, pt, n_global, k, off, tau, starts, chunked)
        torch.cuda.synchronize()
        assert torch.equal(chunked, whole), data


@pytest.mark.parametrize("nq,n,d,data", [
    (2048, 1_250_000, 768, "gauss"),   # a one-GPU group chunk / the W = 8 shard: the top-r sample pass
    (512, 400_000, 768, "int"),        # heavy ties
    (300, 200_000, 128, "gauss"),      # partial query blocks, narrow rows
])
def test_top_r_sample_pass_lower_bounds_the_rth_sampled_key(dev, nq, n, d, data):
    """White-box (round 6): the grouped sample pass keeps per-lane lists of the best sampled keys
    (SCAN_TOPR) instead of writing every sampled score.  The returned [nq, r] list must be sorted, made
    of real sampled keys (each at least as far down the order as the exact r best: element-wise >= in
    key order, so tau can only be lower -- never a wrong result, the filter's counts certify) and equal
    to the exact best-r sampled keys for nearly every query."""
    import torch
    from denseretrievaltoolkits_amd import kernels
    rng = np.random.default_rng(nq + n)
    k = 1000
    q = gauss_bf16(rng, (nq, d)) if data == "gauss" else int_bf16(rng, (nq, d), -4, 4)
    qt = to_dev_bf16(q, dev)
    if data == "gauss":
        pt = torch.randn((n, d), generator=torch.Generator(device=dev).manual_seed(n), device=dev).to(torch.bfloat16)
    else:
        from helpers import device_int_corpus
        pt = device_int_corpus(n, d, -4, 4, seed=n, device=dev)
    n_global = 8 * n
    got = kernels.dist_sample(qt, pt, n_global, k).cpu().numpy().view(np.uint32)
    plan = orc.dist_plan(n, n_global, k)
    r = plan["r"]
    rows = torch.from_numpy(plan["rows"]).to(dev)
    ps = pt[rows].double().cpu().numpy()   # the sampled rows; their exact scores, rounded to fp32
    want = np.sort(orc.desc_key((q.astype(np.float64) @ ps.T).astype(np.float32)), axis=1)[:, :r]
    assert got.shape == (nq, r)
    assert (np.diff(got.astype(np.int64), axis=1) >= 0).all()
    if data == "int":     # exact scores: the lists are comparable key for key
        assert (got >= want).all()
        assert (got == want).all(axis=1).mean() >= 0.99
    else:                 # fp32 chains vs fp64-rounded sums: compare the thresholds' scores within 1e-3
        gt = orc.desc_key_to_score(got[:, r - 1]).astype(np.float64)
        wt = orc.desc_key_to_score(want[:, r - 1]).astype(np.float64)
        assert (gt <= wt + 1e-3).all()
        assert (np.abs(gt - wt) <= 1e-3).mean() >= 0.99
