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


def _np_stats(p):
    """oracle restatement of drt_row_stats_bf16: (max ||p||^2, integer flag, max prefix ||p_[0,32(t+1))||^2)."""
    p64 = p.astype(np.float64)
    nb = (p.shape[1] + 31) // 32
    pref = np.stack([(p64[:, : 32 * (t + 1)] ** 2).sum(1).max() for t in range(nb)])
    return (p64 ** 2).sum(1).max(), float((p == np.rint(p)).all()), pref


def _np_eps(q, p):
    """The scan's certified fp32 error bound per query (csrc/search.hip "Error bound", refine_eps):
    10 u (1 + 1e-3) (sum_{t=1}^{T-1} ||q_[0,32t)|| max ||p_[0,32t)|| + ||q|| max ||p||)."""
    _, _, pref = _np_stats(p)
    q64 = q.astype(np.float64)
    nb = len(pref)
    acc = np.sqrt((q64 ** 2).sum(1) * pref[-1])
    for t in range(1, nb):
        acc += np.sqrt((q64[:, : 32 * t] ** 2).sum(1) * pref[t - 1])
    return 10.0 * 2.0 ** -24 * 1.001 * acc


def test_row_stats_vs_numpy(dev):
    import torch
    from denseretrievaltoolkits_amd import _native, kernels
    rng = np.random.default_rng(1)
    p = gauss_bf16(rng, (10007, 320))
    p[17, :40] *= 3.0   # a row whose PREFIX norm is the largest, not its total
    p = orc.bf16_round(p)
    st = kernels.row_stats(to_dev_bf16(p, dev)).cpu().numpy()
    assert st.shape == (_native.ROW_STATS_LEN,)
    sq, flag, pref = _np_stats(p)
    assert abs(st[0] - sq) <= 1e-4 * sq and st[1] == 0.0
    np.testing.assert_allclose(st[2: 2 + len(pref)], pref, rtol=1e-4)
    assert (st[2 + len(pref):] == 0).all()
    pi = int_bf16(rng, (5000, 320), -4, 4)
    st2 = kernels.row_stats(to_dev_bf16(pi, dev)).cpu().numpy()
    assert st2[1] == 1.0 and abs(st2[0] - (pi.astype(np.float64) ** 2).sum(1).max()) <= 1e-3
    # appended rows combine with the earlier statistics
    both = kernels.row_stats(to_dev_bf16(p[:100], dev), prev=torch.from_numpy(st2).to(dev)).cpu().numpy()
    assert both[1] == 0.0 and both[0] == max(st2[0], np.float32(both[0]))
    np.testing.assert_allclose(both[2:12], np.maximum(st2[2:12], _np_stats(p[:100])[2]), rtol=1e-4)


def _bound_cases(rng):
    """(name, q, p): data that pushes the scan's fp32 error toward the bound."""
    d = 768
    yield "gauss", gauss_bf16(rng, (64, d)), gauss_bf16(rng, (30000, d))
    # the C2 tower's regime: a large common component, every product positive
    yield "common", orc.bf16_round(1.0 + 0.01 * rng.standard_normal((64, d))), \
        orc.bf16_round(1.0 + 0.01 * rng.standard_normal((30000, d)))
    # every k-step drops 31-32 products just under the MFMA's alignment cut (2^-26 below the
    # accumulator): the truncation worst case, with Cauchy-Schwarz tight (q ~ p)
    eps_v = orc.bf16_round(np.float32(2.0 ** -13 * 0.99))
    big = orc.bf16_round(1.0 + rng.integers(0, 64, size=(30000, 1)) / 128.0)
    p = np.full((30000, d), eps_v, np.float32)
    p[:, :1] = big
    q = np.full((16, d), eps_v, np.float32)
    q[:, 0] = 1.0
    yield "truncation", q, orc.bf16_round(p)
    # exponents spread over 16 binades, mixed signs
    yield "spread", orc.bf16_round(rng.standard_normal((64, d)) * np.exp2(rng.integers(-8, 9, size=(64, d)))), \
        orc.bf16_round(rng.standard_normal((30000, d)) * np.exp2(rng.integers(-8, 9, size=(30000, d))))


def test_scan_fp32_error_within_certified_bound(dev):
    """The canonical stage is only as good as its bound: the filter scan's fp32 score of every returned
    row lies within eps (refine_eps) of its exact (fp64) inner product, on data built to approach the
    bound (truncated alignment inside each MFMA step, C-S-tight partial sums)."""
    from denseretrievaltoolkits_amd import kernels
    rng = np.random.default_rng(2024)
    worst = {}
    for name, q, p in _bound_cases(rng):
        qt, pt = to_dev_bf16(q, dev), to_dev_bf16(p, dev)
        s, i, st = kernels.ip_topk(qt, pt, 256)
        s, i = s.cpu().numpy().astype(np.float64), i.cpu().numpy()
        exact = np.einsum("qd,qkd->qk", q.astype(np.float64), p.astype(np.float64)[i])
        ratio = np.abs(s - exact) / _np_eps(q, p)[:, None]
        worst[name] = float(ratio.max())
        assert (ratio <= 1.0).all(), (name, worst)
    assert worst["truncation"] > 0.3, worst   # the case really exercises the truncation term


def test_exact_order_truncation_case_bit_exact(dev):
    """The truncation-worst-case data through the product index: canonical ids equal the fp64 oracle."""
    from denseretrievaltoolkits_amd import search as srch
    rng = np.random.default_rng(7)
    name, q, p = [c for c in _bound_cases(rng) if c[0] == "truncation"][0]
    idx = srch.FlatIPIndex.from_rows(to_dev_bf16(p, dev))
    s, i = idx.search(q, 500)
    es, ei = orc.ip_topk(q, p, 500)
    np.testing.assert_array_equal(i, ei)
    assert idx.order_uncertified == 0


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


def test_exact_order_window_wider_than_list_resolved_wide(dev):
    """Massive exact ties on non-integer values (every row identical, values k + 0.5): the near-tie
    window holds every row, more than the kc candidates -> status 2 (not a rescan: bit 0 clear); the
    wide resolve collects the window, ranks it by exact score and id and clears the bit."""
    import torch
    from denseretrievaltoolkits_amd import kernels
    rng = np.random.default_rng(8)
    n, d, k = 12000, 128, 500          # n <= cap: the dense path (every row scored)
    row = orc.bf16_round(int_bf16(rng, (1, d), -3, 3) + 0.5)
    p = np.repeat(row, n, axis=0)
    q = orc.bf16_round(int_bf16(rng, (4, d), -3, 3) + 0.25)
    qt, pt = to_dev_bf16(q, dev), to_dev_bf16(p, dev)
    stats = kernels.row_stats(pt)
    s, i, st = kernels.ip_topk(qt, pt, k, resolve=False, stats=stats)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 2).all(), st
    assert kernels.resolve_wide(qt, pt, k, 0, s, i, st, stats) == 4
    es, ei = orc.ip_topk(q, p, k)
    np.testing.assert_array_equal(i.cpu().numpy(), ei)
    np.testing.assert_array_equal(s.cpu().numpy(), es)
    assert (st.cpu().numpy() == 0).all()


def test_exact_order_window_beyond_wide_cap(dev):
    """More near-tied rows than the wide resolve can rank (65536 per query): round 6 takes the range-by-range
    exact top-k (kernels.exact_by_ranges) for those queries -- ids and scores == the fp64 order, nothing left
    in the fp32 order.  The rows differ only below the fp32 resolution of their scores (helpers.massive_near_ties)."""
    from helpers import massive_near_ties
    from denseretrievaltoolkits_amd import search as srch
    q, p = massive_near_ties(70000, 64, seed=9)
    k = 10
    idx = srch.FlatIPIndex.from_rows(to_dev_bf16(p, dev))
    s, i = idx.search(q, k)
    es, ei = orc.ip_topk(q, p, k, dtype=np.float64, out_dtype=np.float64)
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(s, es.astype(np.float32))
    assert idx.order_uncertified == 0 and idx.wide_resolved == 2 and idx.range_resolved == 2


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


@pytest.mark.parametrize("grouped", [False, True])
def test_exact_order_degenerate_near_ties_bit_exact(dev, grouped):
    """Sampled path, every score within the fp32 resolution of the others (a common large component +
    1e-4-scale rest: ~76 rows per fp32 ulp of the scores, the untrained-tower regime): the near-tie
    window is far wider than the candidate list, so the product index runs the wide resolve (a filter
    pass at s_k - 2 eps, exact sums, exact-key selection) and the ids equal the fp64 oracle's -- per
    batch and through the grouped path."""
    import torch
    from denseretrievaltoolkits_amd import kernels
    from denseretrievaltoolkits_amd import search as srch
    rng = np.random.default_rng(21)
    n, d, k, nq = 60000, 128, 1000, 4
    p = orc.bf16_round(1e-4 * rng.standard_normal((n, d)))
    p[:, 0] = 8.0
    q = orc.bf16_round(rng.standard_normal((nq, d)))
    q[:, 0] = 8.0
    qt, pt = to_dev_bf16(q, dev), to_dev_bf16(p, dev)
    _, _, st = kernels.ip_topk(qt, pt, k, resolve=False, stats=kernels.row_stats(pt))
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 2).all(), st          # uncertifiable from the candidate list
    idx = srch.FlatIPIndex.from_rows(pt)
    saved = srch.GROUP_MIN_ROWS
    srch.GROUP_MIN_ROWS = 0 if grouped else 1 << 62
    try:
        res = idx.search_batches([qt[:2], qt[2:]], k, id_offset=5)
        torch.cuda.synchronize()
    finally:
        srch.GROUP_MIN_ROWS = saved
    es, ei = orc.ip_topk(q, p, k, id_offset=5)
    np.testing.assert_array_equal(torch.cat([r[1] for r in res]).cpu().numpy(), ei)
    _assert_scores(torch.cat([r[0] for r in res]).cpu().numpy(), es)
    assert idx.order_uncertified == 0 and idx.wide_resolved == nq


@pytest.mark.parametrize("row_offset", [0, 5000])
def test_refine_delta_local_equals_sharded(dev, row_offset):
    """drt_refine_delta_local_bf16 (one shard holds every candidate: the one-GPU grouped search) writes
    the same deltas, window sizes and status as the sharded entry, on Gaussian rows with a candidate list
    of width refine_width(k); candidates outside [row_offset, row_offset + n) get delta 0 in both."""
    import torch
    from denseretrievaltoolkits_amd import kernels, ops
    rng = np.random.default_rng(71 + row_offset)
    nq, n, d, k = 96, 20000, 768, 200
    q = to_dev_bf16(gauss_bf16(rng, (nq, d)), dev)
    p = to_dev_bf16(gauss_bf16(rng, (n, d)), dev)
    kc = kernels.refine_width(k)
    cs, ci = (q.float() @ p.float().T).topk(kc, dim=1)
    ci = ci + row_offset
    if row_offset:   # a few candidates another shard would own
        ci[:, -3:] = row_offset + n + 7
    stats = kernels.row_stats(p)
    drt = ops.load()
    outs = []
    for local in (False, True):
        st = torch.zeros(nq, dtype=torch.int32, device=dev)
        delta, cnt = drt.refine_delta(q, p, row_offset, cs.contiguous(), ci.contiguous(), k, stats, None, st, local)
        torch.cuda.synchronize()
        outs.append((delta.cpu(), cnt.cpu(), st.cpu()))
    (d0, c0, s0), (d1, c1, s1) = outs
    assert torch.equal(c0, c1) and torch.equal(s0, s1)
    win = c0[:, 0]
    for qi in range(nq):   # deltas are defined inside each query's window
        w = int(win[qi])
        if w > 0:
            assert torch.equal(d0[qi, :w], d1[qi, :w]), qi
    assert (win > 0).any()


def test_reset_drops_row_statistics(dev):
    """(round-4 advisor) reset() must drop the row statistics: an index searched over integer rows (exact
    fp32 scores: the integer flag lets the canonical stage skip the near-tie window), reset and refilled
    with at least as many Gaussian rows of larger norm, must rescan them -- ids equal the fp64 oracle."""
    import torch
    from helpers import oracle_topk_streamed
    from denseretrievaltoolkits_amd.search import FlatIPIndex
    rng = np.random.default_rng(97)
    nq, n, d, k = 32, 30000, 768, 100
    idx = FlatIPIndex(d, device=dev)
    idx.add(to_dev_bf16(int_bf16(rng, (n, d), -1, 1), dev))
    qi = int_bf16(rng, (nq, d), -1, 1)
    s0, _ = idx.search_device(to_dev_bf16(qi, dev), k)
    torch.cuda.synchronize()
    st0 = idx.row_stats().cpu().numpy()
    assert st0[1] == 1.0   # integer rows
    idx.reset()
    p = gauss_bf16(rng, (n + 5000, d)) * 3.0
    pd = to_dev_bf16(p, dev)
    idx.add(pd)
    st1 = idx.row_stats().cpu().numpy()
    assert st1[1] == 0.0 and st1[0] > st0[0]
    q = gauss_bf16(rng, (nq, d))
    s, i = idx.search_device(to_dev_bf16(q, dev), k)
    torch.cuda.synchronize()
    es, ei = oracle_topk_streamed(q, pd, k, exact=True)
    np.testing.assert_array_equal(i.cpu().numpy(), ei)
