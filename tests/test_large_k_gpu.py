"""GPU: top-k beyond the candidate-list kernels' 2048 (kernels.ip_topk -> drt_ip_topk_large).

faiss IndexFlatIP answers any k and the reference's ``retrieve_num`` is a free flag
(DRT/arguments.py:195, searched at DRT/trainer/trainer.py:296-297 through
DRT/evaluator/index.py:31-33).  The large-k path always returns the canonical order: ids equal
to the fp64 oracle's (oracle/search_oracle.ip_topk, ties by ascending id) and scores = the exact
sums rounded to fp32 -- on Gaussian data (the threshold from C disjoint row ranges), on
tie-heavy integer data, with fewer rows than k (padded with -1 like faiss) and through
FlatIPIndex's batch paths (which would otherwise group the search).
"""
import numpy as np
import pytest

from helpers import gauss_bf16, int_bf16, to_dev_bf16
from oracle import search_oracle as orc

pytestmark = pytest.mark.gpu


def _large(dev, q, p, k, id_offset=0, with_stats=False):
    import torch
    from denseretrievaltoolkits_amd import kernels
    qt, pt = to_dev_bf16(q, dev), to_dev_bf16(p, dev)
    stats = kernels.row_stats(pt) if with_stats else None
    s, i, st = kernels.ip_topk(qt, pt, k, id_offset=id_offset, stats=stats)
    torch.cuda.synchronize()
    return s.cpu().numpy(), i.cpu().numpy(), st.cpu().numpy()


def _assert_scores(gs, es):
    """fp32 roundings of the same exact sum computed in two fp64 orders: equal up to one fp32 ulp."""
    ulp = np.spacing(np.abs(es).astype(np.float32))
    assert (np.abs(gs.astype(np.float64) - es.astype(np.float64)) <= ulp).all()
    assert (gs == es).mean() > 0.999


@pytest.mark.parametrize("nq,n,d,k,stats", [
    (20, 200000, 768, 5000, False),    # threshold from 3 row ranges (m = 1667), BERT-base width
    (130, 90000, 256, 2049, True),     # k just past the list kernels, 2 query chunks of 128
    (3, 30000, 128, 4096, False),      # n <= 65536: every row collected
    (4, 150000, 64, 32768, False),     # k at its maximum (16 row ranges of 2048)
    (3, 60000, 128, 32768, True),      # k > n / 2: the selected scores cross zero (rank bins on the score)
])
def test_large_k_gaussian_bit_exact(dev, nq, n, d, k, stats):
    rng = np.random.default_rng(nq + n + d + k)
    q = gauss_bf16(rng, (nq, d))
    p = gauss_bf16(rng, (n, d))
    gs, gi, st = _large(dev, q, p, k, id_offset=11, with_stats=stats)
    es, ei = orc.ip_topk(q, p, k, id_offset=11)
    assert (st == 0).all()
    np.testing.assert_array_equal(gi, ei)
    _assert_scores(gs, es)


def test_large_k_integer_ties_by_id(dev):
    """Small integers: massive exact ties, resolved by ascending id (scores exact in fp32)."""
    rng = np.random.default_rng(5)
    q = int_bf16(rng, (6, 64), -2, 2)
    p = int_bf16(rng, (60000, 64), -2, 2)
    gs, gi, st = _large(dev, q, p, 3000)
    es, ei = orc.ip_topk(q, p, 3000)
    np.testing.assert_array_equal(gi, ei)
    np.testing.assert_array_equal(gs, es)


def test_large_k_fewer_rows_than_k_pads(dev):
    rng = np.random.default_rng(7)
    q = int_bf16(rng, (3, 64))
    p = int_bf16(rng, (2500, 64))
    gs, gi, st = _large(dev, q, p, 4000, id_offset=100)
    es, ei = orc.ip_topk(q, p, 4000, id_offset=100)
    np.testing.assert_array_equal(gi, ei)
    np.testing.assert_array_equal(gs, es)
    assert (gi[:, 2500:] == -1).all() and (gs[:, 2500:] == orc.PAD_SCORE).all()
    gs, gi, st = _large(dev, q, np.zeros((0, 64), np.float32), 4000)   # an empty shard
    assert (gi == -1).all() and (gs == orc.PAD_SCORE).all() and (st == 0).all()


def test_large_k_limits(dev):
    import torch
    from denseretrievaltoolkits_amd import kernels
    q = torch.zeros((2, 64), dtype=torch.bfloat16, device=dev)
    p = torch.zeros((10, 64), dtype=torch.bfloat16, device=dev)
    with pytest.raises(ValueError):
        kernels.ip_topk(q, p, 32769)
    # 70,000 rows inside one fp32 error bound of each other: more than the 65,536 a query may collect ->
    # round 6: the range-by-range exact top-k (kernels.exact_by_ranges) gives the fp64 order anyway
    from helpers import massive_near_ties
    qn, pn = massive_near_ties(70000, 64, seed=4)
    s, i, st = kernels.ip_topk(torch.from_numpy(qn).to(dev).bfloat16(), torch.from_numpy(pn).to(dev).bfloat16(), 3000)
    es, ei = orc.ip_topk(qn, pn, 3000, dtype=np.float64, out_dtype=np.float64)
    np.testing.assert_array_equal(i.cpu().numpy(), ei)
    np.testing.assert_array_equal(s.cpu().numpy(), es.astype(np.float32))
    assert (st.cpu().numpy() == 0).all()


def test_flat_index_large_k_batches(dev):
    """FlatIPIndex at a grouped-path size: k > 2048 takes the per-batch large-k path in search,
    search_batches and enqueue_batches, equal to the fp64 oracle."""
    import torch
    from denseretrievaltoolkits_amd import search as srch
    rng = np.random.default_rng(31)
    q = gauss_bf16(rng, (24, 128))
    p = gauss_bf16(rng, (520000, 128))
    k = 2500
    es, ei = orc.ip_topk(q, p, k)
    idx = srch.FlatIPIndex.from_rows(to_dev_bf16(p, dev))
    assert idx._use_groups(1000) and not idx._use_groups(k)
    qd = to_dev_bf16(q, dev)
    res = idx.search_batches([qd[a: a + 8] for a in range(0, 24, 8)], k)
    np.testing.assert_array_equal(torch.cat([r[1] for r in res]).cpu().numpy(), ei)
    _assert_scores(torch.cat([r[0] for r in res]).cpu().numpy(), es)
    pend = idx.enqueue_batches([qd[:8]], k)
    s, i = idx.finish_batch(pend[0])
    np.testing.assert_array_equal(i.cpu().numpy(), ei[:8])
    s, i = idx.search(q[8:16], k)
    np.testing.assert_array_equal(i, ei[8:16])
    assert idx.order_uncertified == 0
    # caller-owned output buffers (search_batches' per-batch path), and an index without the exact order
    outs = [(torch.empty((8, k), dtype=torch.float32, device=dev), torch.empty((8, k), dtype=torch.int64, device=dev))]
    res = idx.search_batches([qd[16:24]], k, outs=outs)
    assert res[0][1].data_ptr() == outs[0][1].data_ptr()
    np.testing.assert_array_equal(outs[0][1].cpu().numpy(), ei[16:24])
    idx.exact_order = False
    s, i = idx.search_device(qd[:8], k)
    np.testing.assert_array_equal(i.cpu().numpy(), ei[:8])


def test_large_k_corpus_ordered_by_relevance(dev):
    """A corpus whose first third is relevant to the queries (passages grouped by article, sources
    appended one after another): the range plan's minimum is dragged down by the weak ranges and every
    row of the first range passes it (> 65,536 rows), so those queries are retried at a threshold next
    to their own k-th score (kernels._kth_bound) -- the answer is still the fp64 oracle's."""
    rng = np.random.default_rng(41)
    n, d, k, nq = 200000, 768, 5000, 6
    base = rng.standard_normal((1, d)).astype(np.float32)
    q = gauss_bf16(rng, (nq, d)) * 0.25 + base
    p = rng.standard_normal((n, d)).astype(np.float32)
    p[: n // 3] += 0.5 * base           # rows [0, n / 3) score far above the rest
    from oracle.search_oracle import bf16_round
    q, p = bf16_round(q), bf16_round(p)
    gs, gi, st = _large(dev, q, p, k)
    es, ei = orc.ip_topk(q, p, k)
    assert (st == 0).all()
    assert (ei < n // 3).all()          # the setting: the whole top-k comes from the first range
    np.testing.assert_array_equal(gi, ei)
    _assert_scores(gs, es)


def test_exact_keys_and_merge_exact_vs_oracle(dev):
    """The sharded k > 2048 pieces (round 6): kernels.ip_topk_exact_keys returns each shard's canonical
    top-k with its exact order keys (integer rows: the fp64 sums are exact, so the keys equal the
    oracle's bit for bit), and kernels.merge_exact merges [nparts, nq, k] lists by (key, global id) into
    the single index's top-k."""
    import torch
    from denseretrievaltoolkits_amd import kernels
    rng = np.random.default_rng(9)
    q = int_bf16(rng, (4, 64), -3, 3)
    p = int_bf16(rng, (50000, 64), -3, 3)
    k, bounds = 2500, [(0, 16000), (16000, 16000), (16000, 50000)]   # an empty shard too
    qt = to_dev_bf16(q, dev)
    keys, ids = [], []
    for a, b in bounds:
        kk, ii = kernels.ip_topk_exact_keys(qt, to_dev_bf16(p[a:b], dev), k, id_offset=a)
        ek, ei = orc.exact_keys_topk(q, p[a:b], k, id_offset=a)
        np.testing.assert_array_equal(ii.cpu().numpy(), ei)
        np.testing.assert_array_equal(kk.cpu().numpy().view(np.uint64), ek)
        keys.append(kk)
        ids.append(ii)
    s, i = kernels.merge_exact(torch.stack(keys), torch.stack(ids), k)
    es, ei = orc.ip_topk(q, p, k)
    np.testing.assert_array_equal(i.cpu().numpy(), ei)
    np.testing.assert_array_equal(s.cpu().numpy(), es)
    # random sorted lists with ragged fills (pads last), ties across parts broken by id
    nparts, nq = 5, 3
    kr = orc.desc_key64(rng.integers(-3000, 3000, size=(nparts, nq, k)).astype(np.float64) / 8.0)
    ir = rng.permutation(nparts * nq * k).reshape(nparts, nq, k).astype(np.int64)
    for l in range(nparts):
        for r in range(nq):
            o = np.lexsort((ir[l, r], kr[l, r]))
            kr[l, r], ir[l, r] = kr[l, r][o], ir[l, r][o]
            c = int(rng.integers(0, k + 1))
            kr[l, r, c:], ir[l, r, c:] = orc.PAD_KEY64, -1
    s, i = kernels.merge_exact(torch.from_numpy(kr.view(np.int64)).to(dev), torch.from_numpy(ir).to(dev), k)
    es, ei = orc.merge_exact(kr, ir, k)
    np.testing.assert_array_equal(i.cpu().numpy(), ei)
    np.testing.assert_array_equal(s.cpu().numpy(), es)
