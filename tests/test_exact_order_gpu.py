"""GPU: the canonical exact-score order (kernels.refine; include/drt.h "Canonical order").

The scan ranks rows by fp32 sums of bf16 products; on real-valued data rows whose exact inner
products are closer than the fp32 summation error come out in MFMA order.  With the row
statistics the product path re-ranks every query's near-tie window by the EXACT products (fp64
sums), so the ids must equal the fp64 oracle's (oracle/search_oracle.ip_topk: numpy float64,
ties by ascending id) BIT FOR BIT on Gaussian data too -- north_star's "bit-exact retrieved
doc-ids / ranks" -- and the scores are the exact sums rounded to fp32 (the oracle's scores up to
the last fp64 bit).  Reference: BaseFaissIPRetriever.search (DRT/evaluator/index.py:31-33).
"""
import numpy as np
import pytest

from helpers import gauss_bf16, int_bf16, sample_plan, to_dev_bf16
from oracle import search_oracle as orc

pytestmark = pytest.mark.gpu


def _exact(dev, q, p, k, id_offset=0, resolve=True):
    import torch
    from denseretrievaltoolkits_amd import kernels
    qt, pt = to_dev_bf16(q, dev), to_dev_bf16(p, dev)
    stats = kernels.row_stats(pt)
    s, i, st = kernels.ip_topk(qt, pt, k, id_offset=id_offset, resolve=resolve, stats=stats)
    torch.cuda.synchronize()
    return s.cpu().numpy(), i.cpu().numpy(), st.cpu().numpy()


def _assert_scores(gs, es):
    """fp32 roundings of the same exact sum computed in two fp64 orders: equal up to one fp32 ulp."""
    ulp = np.spacing(np.abs(es).astype(np.float32))
    assert (np.abs(gs.astype(np.float64) - es.astype(np.float64)) <= ulp).all()
    assert (gs == es).mean() > 0.999


def test_row_stats_vs_numpy(dev):
    import torch
    from denseretrievaltoolkits_amd import kernels
    rng = np.random.default_rng(1)
    p = gauss_bf16(rng, (10007, 320))
    st = kernels.row_stats(to_dev_bf16(p, dev)).cpu().numpy()
    sq = (p.astype(np.float64) ** 2).sum(1).max()
    assert abs(st[0] - sq) <= 1e-4 * sq and st[1] == 0.0
    pi = int_bf16(rng, (5000, 320), -4, 4)
    st2 = kernels.row_stats(to_dev_bf16(pi, dev)).cpu().numpy()
    assert st2[1] == 1.0 and abs(st2[0] - (pi.astype(np.float64) ** 2).sum(1).max()) <= 1e-3
    # appended rows combine with the earlier statistics
    both = kernels.row_stats(to_dev_bf16(p[:100], dev), prev=torch.from_numpy(st2).to(dev)).cpu().numpy()
    assert both[1] == 0.0 and both[0] == max(st2[0], np.float32(both[0]))


@pytest.mark.parametrize("nq,n,d,k", [
    (128, 120000, 768, 1000),   # sampled threshold path, the headline shape at a small n
    (37, 9000, 768, 100),       # dense small-shard path (n <= cap)
    (16, 300000, 256, 1500),    # wider k (kc = 1875)
    (5, 50000, 1024, 10),       # d = 1024, tiny k
])
def test_exact_order_gaussian_bit_exact(dev, nq, n, d, k):
    rng = np.random.default_rng(nq + n + d + k)
    q = gauss_bf16(rng, (nq, d))
    p = gauss_bf16(rng, (n, d))
    gs, gi, st = _exact(dev, q, p, k, id_offset=7)
    es, ei = orc.ip_topk(q, p, k, id_offset=7)
    assert (st == 0).all(), st
    np.testing.assert_array_equal(gi, ei)
    _assert_scores(gs, es)


def test_exact_order_fixes_what_fp32_order_swaps(dev):
    """The same inputs through the fp32 scan order differ from the fp64 oracle (near-ties in MFMA
    order) -- the canonical stage is what makes them equal."""
    import torch
    from denseretrievaltoolkits_amd import kernels
    rng = np.random.default_rng(99)
    q = gauss_bf16(rng, (128, 768))
    p = gauss_bf16(rng, (200000, 768))
    es, ei = orc.ip_topk(q, p, 1000)
    qt, pt = to_dev_bf16(q, dev), to_dev_bf16(p, dev)
    _, i32, _ = kernels.ip_topk(qt, pt, 1000)
    _, iex, st = kernels.ip_topk(qt, pt, 1000, stats=kernels.row_stats(pt))
    torch.cuda.synchronize()
    assert (i32.cpu().numpy() != ei).any(), "expected fp32 near-tie swaps on 128 x 200k Gaussian queries"
    np.testing.assert_array_equal(iex.cpu().numpy(), ei)
    assert (st.cpu().numpy() == 0).all()


@pytest.mark.parametrize("nq,n,d,k", [(128, 50000, 768, 1000), (1, 200003, 768, 1000), (9, 20000, 128, 2048)])
def test_exact_order_integer_unchanged(dev, nq, n, d, k):
    """Integer-valued rows and queries are scored exactly in fp32: the stage keeps the fp32 order
    (eps = 0), bit-exact as before, also at k = 2048 where the window has no room."""
    rng = np.random.default_rng(3 * nq + n)
    q = int_bf16(rng, (nq, d), -4, 4)
    p = int_bf16(rng, (n, d), -4, 4)
    gs, gi, st = _exact(dev, q, p, k)
    es, ei = orc.ip_topk(q, p, k)
    assert (st == 0).all()
    np.testing.assert_array_equal(gi, ei)
    np.testing.assert_array_equal(gs, es)


def test_exact_order_resolve_path(dev):
    """An uncertified query (sample threshold too high) is rescanned densely and re-ranked
    exactly: Gaussian rows, the sampled rows made the strongest."""
    import torch
    from denseretrievaltoolkits_amd import kernels
    rng = np.random.default_rng(5)
    n, d, k, nq = 60000, 128, 1000, 3
    plan = sample_plan(n, k)
    q = np.abs(gauss_bf16(rng, (nq, d)))
    p = gauss_bf16(rng, (n, d))
    p[plan["rows"]] = orc.bf16_round(np.abs(p[plan["rows"]]) + 3.0)
    qt, pt = to_dev_bf16(q, dev), to_dev_bf16(p, dev)
    stats = kernels.row_stats(pt)
    s, i, st = kernels.ip_topk(qt, pt, k, resolve=False, stats=stats)
    torch.cuda.synchronize()
    assert ((st.cpu().numpy() & 1) != 0).all()
    assert kernels.resolve_failed(qt, pt, k, 0, s, i, st, stats=stats) == nq
    es, ei = orc.ip_topk(q, p, k)
    np.testing.assert_array_equal(i.cpu().numpy(), ei)
    _assert_scores(s.cpu().numpy(), es)
    assert (st.cpu().numpy() == 0).all()


def test_exact_order_window_wider_than_list_keeps_fp32_order(dev):
    """Massive exact ties on non-integer values (every row identical, values k + 0.5): the
    near-tie window holds every row, more than the kc candidates -> status bit 1, the fp32 order
    (here: ascending id, all scores equal) is kept, and nothing is rescanned (bit 0 clear)."""
    rng = np.random.default_rng(8)
    n, d, k = 12000, 128, 500          # n <= cap: the dense path (every row scored)
    row = orc.bf16_round(int_bf16(rng, (1, d), -3, 3) + 0.5)
    p = np.repeat(row, n, axis=0)
    q = orc.bf16_round(int_bf16(rng, (4, d), -3, 3) + 0.25)
    gs, gi, st = _exact(dev, q, p, k, resolve=False)
    assert ((st & 2) != 0).all() and ((st & 1) == 0).all(), st
    es, ei = orc.ip_topk(q, p, k)
    np.testing.assert_array_equal(gi, ei)
    np.testing.assert_array_equal(gs, es)


def test_flat_index_exact_order_default_and_counter(dev):
    """FlatIPIndex (BaseFaissIPRetriever's index) ranks canonically by default; the per-batch and
    grouped batch paths agree bit for bit with the fp64 oracle, and nothing is left uncertified."""
    import torch
    from denseretrievaltoolkits_amd import search as srch
    rng = np.random.default_rng(21)
    q = gauss_bf16(rng, (96, 768))
    p = gauss_bf16(rng, (150000, 768))
    es, ei = orc.ip_topk(q, p, 1000)
    idx = srch.FlatIPIndex.from_rows(to_dev_bf16(p, dev))
    assert idx.exact_order
    qd = to_dev_bf16(q, dev)
    for gmin in (1 << 62, 0):   # per-batch path, then the grouped path
        saved = srch.GROUP_MIN_ROWS
        srch.GROUP_MIN_ROWS = gmin
        try:
            res = idx.search_batches([qd[a: a + 32] for a in range(0, 96, 32)], 1000)
            torch.cuda.synchronize()
        finally:
            srch.GROUP_MIN_ROWS = saved
        np.testing.assert_array_equal(torch.cat([r[1] for r in res]).cpu().numpy(), ei)
        _assert_scores(torch.cat([r[0] for r in res]).cpu().numpy(), es)
    assert idx.order_uncertified == 0 and idx.group_fallbacks == 0


def test_exact_order_degenerate_near_ties_keep_fp32_result_without_rescan(dev):
    """Sampled path, every score within the fp32 error bound of every other (a common large
    component + 1e-4-scale rest: the untrained-tower case of the C2 leg): the near-tie window
    reaches below the filter threshold, so the canonical order cannot be certified from the list.
    Status bit 1 is set, bit 0 is NOT (no dense rescan), and the result is exactly the fp32 path's
    (ip_topk without row statistics): the certified fp32 top-k in the fp32 order."""
    import torch
    from denseretrievaltoolkits_amd import kernels
    rng = np.random.default_rng(21)
    n, d, k, nq = 60000, 128, 1000, 4
    p = orc.bf16_round(1e-4 * rng.standard_normal((n, d)))
    p[:, 0] = 8.0
    q = orc.bf16_round(rng.standard_normal((nq, d)))
    q[:, 0] = 8.0
    qt, pt = to_dev_bf16(q, dev), to_dev_bf16(p, dev)
    stats = kernels.row_stats(pt)
    s, i, st = kernels.ip_topk(qt, pt, k, resolve=False, stats=stats)
    s32, i32, st32 = kernels.ip_topk(qt, pt, k, resolve=False)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    assert ((st & 2) != 0).all() and ((st & 1) == 0).all(), st
    assert (st32.cpu().numpy() == 0).all()
    assert torch.equal(i, i32) and torch.equal(s, s32)
