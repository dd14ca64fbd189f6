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


KC = 1256


def _rec(n, world, grouped, launch_ms, steps=20, group=2048, chunks=None):
    import bench
    a = _args(n, steps)
    per = -(-n // world)
    shapes = bench.launch_shapes(steps, 128, grouped, group, per, chunks)
    traffic = (None, None) if grouped else (15_385_000_000, "r04aw_pmc_traffic.json")
    return bench.search_record(a, world, grouped, group, KC, steps * 2.7e-3, launch_ms * len(shapes), len(shapes),
                               traffic, chunks=chunks)


def test_launch_shapes_group_batches_and_chunks_like_search():
    import bench
    from denseretrievaltoolkits_amd import search as srch
    assert bench.launch_shapes(20, 128, False, 2048, 10_000_000) == [(128, 10_000_000)] * 20
    assert bench.launch_shapes(20, 128, True, 2048, 1_000_000) == [(2048, 1_000_000), (512, 1_000_000)]
    assert bench.launch_shapes(16, 128, True, 2048, 5) == [(2048, 5)]
    assert bench.launch_shapes(3, 128, True, 128, 7) == [(128, 7)] * 3
    ch = srch.group_chunks(10_000_000)
    assert len(ch) == 8 and ch[0] == (0, 1_250_000) and ch[-1][1] == 10_000_000
    assert bench.launch_shapes(16, 128, True, 2048, 10_000_000, ch) == [(2048, 1_250_000)] * 8
    assert srch.group_chunks(1_000_000) == [(0, 1_000_000)]
    assert [b - a for a, b in srch.group_chunks(2_600_000)] == [866_667, 866_667, 866_666]


def test_world1_10m_per_batch_is_hbm_bound_with_survey_bytes():
    r = _rec(10_000_000, 1, False, 2.44)
    rf = r["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s"
    assert rf["alg_bytes_per_launch"] == 10_000_000 * 768 * 2 + 128 * 768 * 2 + 128 * 1000 * 12
    assert rf["launch_shapes"] == [(128, 10_000_000)]
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


def test_world1_10m_grouped_chunks_are_priced_per_chunk_launch():
    from denseretrievaltoolkits_amd import search as srch
    ch = srch.group_chunks(10_000_000)
    r = _rec(10_000_000, 1, True, 3.8, steps=16, chunks=ch)
    rf = r["roofline"]
    assert rf["launches"] == 8 and rf["launch_shapes"] == [(2048, 1_250_000)]
    assert rf["bound"] == "mfma" and abs(rf["frac"] - 2 * 2048 * 1_250_000 * 768 / 2.5e15 / 3.8e-3) < 1e-3
    assert "8 launch(es) over row chunks" in r["config"]["path"]


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
        t_hbm = (per * 768 * 2 + 128 * 768 * 2 + 128 * (KC + 1) * 8) / 8e12
        assert abs(rf["frac"] - t_hbm / 0.30e-3) < 1e-3


def test_world2_grouped_prices_the_shard_chunks():
    """World 2 over 10M rows: each 5M-row shard is filtered in 4 chunk launches (the count of the
    largest shard, the same on every rank)."""
    from types import SimpleNamespace as NS
    from denseretrievaltoolkits_amd import search as srch
    fake = NS(ntotal=10_000_000, world=2, local=NS(ntotal=5_000_000))
    ch = srch.ShardedFlatIP.group_chunks(fake)
    assert ch == [(0, 1_250_000), (1_250_000, 2_500_000), (2_500_000, 3_750_000), (3_750_000, 5_000_000)]
    # a short last shard keeps the count (empty chunks allowed)
    short = srch.ShardedFlatIP.group_chunks(NS(ntotal=10_000_000, world=3, local=NS(ntotal=2)))
    assert len(short) == 3 and short[-1] == (2, 2)
    r = _rec(10_000_000, 2, True, 3.8, steps=16, chunks=ch)
    rf = r["roofline"]
    assert rf["launches"] == 4 and rf["launch_shapes"] == [(2048, 1_250_000)]
    assert "4 launch(es) over row chunks of the shard" in r["config"]["path"]


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bench_corpus_union_of_shards_is_the_world1_corpus(world, monkeypatch):
    """corpus rows are seeded by GLOBAL row block, so the W shards of the 1/2/4/8-GPU
    runs concatenate to the one-GPU corpus (same rows searched at every N)."""
    import torch
    import bench
    monkeypatch.setattr(bench, "CORPUS_BLOCK_ROWS", 1000)
    n, d = 5321, 16
    full, lo, hi = bench.gen_shard(n, 1, 0, d, torch.device("cpu"))
    assert (lo, hi) == (0, n)
    parts = [bench.gen_shard(n, world, r, d, torch.device("cpu")) for r in range(world)]
    assert parts[0][1] == 0 and parts[-1][2] == n
    assert all(parts[r][2] == parts[r + 1][1] for r in range(world - 1))
    assert torch.equal(torch.cat([p[0] for p in parts]).view(torch.int16), full.view(torch.int16))


def test_per_shape_roofline_of_a_20_step_run():
    """The driver's --steps 20 runs a 2048-query group and a 512-query group: the record reports each
    launch shape's own average and fraction beside the mixed average."""
    import bench
    from denseretrievaltoolkits_amd import search as srch
    ch = srch.group_chunks(10_000_000)
    shapes = bench.launch_shapes(20, 128, True, 2048, 10_000_000, ch)
    each = [3.0 if q == 2048 else 0.8 for q, _ in shapes]
    a = _args(10_000_000, 20)
    r = bench.search_record(a, 1, True, 2048, KC, 20 * 1.7e-3, sum(each), len(each), (None, None), chunks=ch,
                            each_ms=each)
    ps = r["roofline"]["per_shape"]
    assert [(p["queries"], p["rows"], p["launches"]) for p in ps] == [(2048, 1_250_000, 8), (512, 1_250_000, 8)]
    assert ps[0]["avg_launch_ms"] == 3.0 and ps[1]["avg_launch_ms"] == 0.8
    assert abs(ps[0]["frac"] - 2 * 2048 * 1_250_000 * 768 / 2.5e15 / 3.0e-3) < 1e-3
    assert r["roofline"]["avg_launch_ms"] == round(sum(each) / 16, 4)
