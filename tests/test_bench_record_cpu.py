"""CPU: bench.py's headline record states the path it timed and prices each filter launch by its own
shape (bytes = N_s d 2 + Q d 2 + the result lists, flops = 2 Q N_s d, t_roof = the larger
of bytes / 8 TB/s and flops / 2.5 PF/s).  The per-batch pass at Q = 128 is HBM-bound; the grouped
launch (Q = 2048, 16 query blocks sharing each tile through L2) is MFMA-side."""
import os
import sys
from types import SimpleNamespace

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _args(n, steps=20):
    return SimpleNamespace(n_corpus=n, dim=768, k=1000, qb=128, steps=steps, warmup=3, protocol="global_tau")


def _rec(n, world, grouped, launch_ms, steps=20, group=2048):
    import bench
    a = _args(n, steps)
    sizes = bench.launch_queries(steps, 128, grouped, group)
    return bench.search_record(a, world, grouped, group, 1512, steps * 2.7e-3, launch_ms * len(sizes), len(sizes),
                               (15_385_000_000, "r04aw_pmc_traffic.json"))


def test_launch_queries_groups_batches_like_search():
    import bench
    assert bench.launch_queries(20, 128, False, 2048) == [128] * 20
    assert bench.launch_queries(20, 128, True, 2048) == [2048, 512]
    assert bench.launch_queries(16, 128, True, 2048) == [2048]
    assert bench.launch_queries(3, 128, True, 128) == [128] * 3


def test_world1_10m_per_batch_is_hbm_bound_with_survey_bytes():
    r = _rec(10_000_000, 1, False, 2.44)
    rf = r["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s"
    assert rf["alg_bytes_per_launch"] == 10_000_000 * 768 * 2 + 128 * 768 * 2 + 128 * 1000 * 12
    assert 0.78 <= rf["frac"] <= 0.80 and rf["frac"] <= 1.0
    assert rf["traffic"] == 15_385_000_000
    assert "per batch" in r["config"]["workload"] and "per batch" in r["config"]["path"]
    assert r["config"]["queries_per_filter_launch"] == 128


def test_world1_1m_grouped_is_mfma_side():
    r = _rec(1_000_000, 1, True, 16 * 0.25, steps=16)
    rf = r["roofline"]
    assert rf["bound"] == "mfma" and rf["unit"] == "TFLOP/s" and rf["peak"] == 2500.0
    assert rf["alg_flops_per_launch"] == 2 * 2048 * 1_000_000 * 768
    assert rf["frac"] <= 1.0 and rf["traffic"] is None
    assert "groups of 2048" in r["config"]["workload"] and r["config"]["queries_per_filter_launch"] == 2048


@pytest.mark.parametrize("grouped,launch_ms,bound", [(True, 3.9, "mfma"), (False, 0.30, "hbm")])
def test_world8_prices_the_launch_it_ran(grouped, launch_ms, bound):
    r = _rec(10_000_000, 8, grouped, launch_ms * (1 if not grouped else 1), steps=16, group=2048 if grouped else 128)
    rf = r["roofline"]
    assert rf["bound"] == bound and 0.0 < rf["frac"] <= 1.0
    per = 1_250_000
    if grouped:
        assert abs(rf["frac"] - 2 * 2048 * per * 768 / 2.5e15 / 3.9e-3) < 1e-3
        assert "ShardedFlatIP" in r["config"]["path"] and "groups of 2048" in r["config"]["workload"]
    else:
        t_hbm = (per * 768 * 2 + 128 * 768 * 2 + 128 * 1513 * 8) / 8e12
        assert abs(rf["frac"] - t_hbm / 0.30e-3) < 1e-3
