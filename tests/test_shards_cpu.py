"""Shard files (shards.py): memory-mapped bf16 rows, rank-ordered file
lists, re-sharding across world sizes, and the gloo multi-rank load -> search path.
The reference writes `{ep}.{rank}.npy` fp32 and has rank 0 concatenate them in
os.listdir order (DRT/trainer/trainer.py:210-216, 223-248); here the order is the rank
number and each rank streams only its own contiguous row range."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from denseretrievaltoolkits_amd import shards
from tests.test_distributed_cpu import _OracleShard, _free_port, _oracle_merge, _oracle_merge_packed


def _rows(n, d, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, d, generator=g).to(torch.bfloat16)


def _write(tmp_path, sizes, d, ep=3):
    parts = [_rows(n, d, 100 + r) for r, n in enumerate(sizes)]
    for r, p in enumerate(parts):
        shards.save_rows(p, shards.shard_path(str(tmp_path), ep, r), chunk_bytes=2 * d * 7)
    return torch.cat(parts, 0)


def test_save_load_roundtrip_bit_exact(tmp_path):
    x = _rows(1001, 64, 0)
    p = str(tmp_path / "a.bf16.npy")
    shards.save_rows(x, p, chunk_bytes=2 * 64 * 13)        # 13-row chunks, ragged tail
    mm = np.load(p, mmap_mode="r")
    assert mm.dtype == np.int16 and mm.shape == (1001, 64)
    for cb in (2 * 64 * 5, 1 << 20):
        y = shards.load_rows([p], 0, 1001, "cpu", chunk_bytes=cb)
        assert torch.equal(y.view(torch.int16), x.view(torch.int16))
    y = shards.load_rows([p], 17, 400, "cpu", chunk_bytes=2 * 64 * 5)
    assert torch.equal(y.view(torch.int16), x[17:400].view(torch.int16))


def test_list_shards_rank_order_and_gaps(tmp_path):
    for r in range(12):
        shards.save_rows(_rows(2, 64, r), shards.shard_path(str(tmp_path), 0, r))
    shards.save_rows(_rows(2, 64, 99), shards.shard_path(str(tmp_path), 1, 0))   # another epoch
    paths = shards.list_shards(str(tmp_path), 0)
    assert [os.path.basename(p) for p in paths] == [f"0.{r}.bf16.npy" for r in range(12)]
    os.remove(shards.shard_path(str(tmp_path), 0, 5))
    with pytest.raises(FileNotFoundError):
        shards.list_shards(str(tmp_path), 0)
    with pytest.raises(FileNotFoundError):
        shards.list_shards(str(tmp_path), 7)


@pytest.mark.parametrize("sizes", [[300, 0, 201, 1], [5], [0, 0, 9], [64, 64, 64, 64]])
@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_reshard_any_world_concatenates_to_the_corpus(tmp_path, sizes, world):
    full = _write(tmp_path, sizes, 64)
    paths = shards.list_shards(str(tmp_path), 3)
    got_sizes, d = shards.shard_sizes(paths)
    assert got_sizes == sizes and d == 64
    n = sum(sizes)
    pieces = []
    for r in range(world):
        a, b = shards.split_rows(n, world, r)
        pieces.append(shards.load_rows(paths, a, b, "cpu", chunk_bytes=2 * 64 * 11))
    cat = torch.cat(pieces, 0)
    assert torch.equal(cat.view(torch.int16), full.view(torch.int16))


def test_bad_files_and_ranges(tmp_path):
    p = str(tmp_path / "f.npy")
    np.save(p, np.zeros((3, 64), np.float32))
    with pytest.raises(ValueError):
        shards.shard_sizes([p])
    q = str(tmp_path / "g.npy")
    shards.save_rows(_rows(4, 64, 1), q)
    with pytest.raises(ValueError):
        shards.plan_reads([4], 0, 5)
    with pytest.raises(ValueError):
        shards.save_rows(torch.zeros(3, 64), q)


def _load_worker(rank, world, port, directory, k, out_q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from denseretrievaltoolkits_amd.search import ShardedFlatIP
    from oracle import search_oracle as orc
    idx = ShardedFlatIP.load_shards(directory, 3, local=_OracleShard(64), merge=_oracle_merge,
                                    merge_packed=_oracle_merge_packed)
    full = np.load(os.path.join(directory, "full.npy"))
    q = np.load(os.path.join(directory, "q.npy"))
    a, b = shards.split_rows(full.shape[0], world, rank)
    ok = idx.offset == a and idx.ntotal == full.shape[0] and np.array_equal(idx.local.rows, full[a:b])
    s, i = idx.search_device(q, k)
    es, ei = orc.ip_topk(q, full, k)
    ok = ok and np.array_equal(i.numpy(), ei) and np.array_equal(s.numpy(), es)
    out_q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_loads_files_from_world3_and_searches(tmp_path):
    """Files written by 3 ranks, loaded by 2: each rank's contiguous range, then the sharded search
    (oracle-injected shard scan) equals the single-index oracle over the whole corpus."""
    full = _write(tmp_path, [700, 0, 333], 64)
    np.save(tmp_path / "full.npy", full.float().numpy())
    np.save(tmp_path / "q.npy", _rows(4, 64, 7).float().numpy())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_load_worker, args=(r, 2, port, str(tmp_path), 25, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] for r in res), res
