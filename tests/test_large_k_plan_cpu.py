"""CPU: the large-k threshold plan (kernels.large_k_ranges): the ranges partition the rows, each
holds at least m rows, m fits the list kernels (<= 2048) and C * m >= k -- so the minimum of the
ranges' m-th scores is a lower bound of the k-th score (drt_ip_topk_large's precondition)."""
import pytest

from denseretrievaltoolkits_amd import kernels


@pytest.mark.parametrize("n", [65537, 70000, 150000, 1_000_003, 10_000_000])
@pytest.mark.parametrize("k", [2049, 3000, 4096, 5000, 16385, 32768])
def test_large_k_ranges_bound_the_kth_score(n, k):
    m, ranges = kernels.large_k_ranges(n, k)
    assert 1 <= m <= kernels.MAX_K
    assert len(ranges) * m >= k
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    assert all(a1 == b0 for (_, b0), (a1, _) in zip(ranges, ranges[1:]))
    assert all(b - a >= m for a, b in ranges)


def test_large_k_small_corpus_collects_every_row():
    assert kernels.large_k_ranges(65536, 4096) is None
    assert kernels.large_k_ranges(10, 4096) is None
