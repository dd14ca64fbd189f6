"""GPU: the device-tensor collectives through a REAL RCCL communicator.

The multi-rank GPU tests (test_multirank_gpu.py) share one GPU between ranks, which RCCL
does not allow, so they run over gloo (payloads staged through host memory).  Here ONE
process initialises an ``nccl`` (= RCCL on ROCm) group of world 1 and turns on comm.py's
test-only forcing, so every collective of the hot path takes its device branch:
``all_gather_into_tensor`` / ``all_reduce`` on HIP tensors inside RCCL.  The sharded
search (both protocols, per batch and grouped) must then equal the oracle bit for bit,
exactly as on a multi-GPU node where the same calls gather the other shards' lists.

Reference: the NCCL process group of run_random_sampling.py:59-61; the exchange it
replaces is the file-system gather of trainer.py:210-262.
"""
import os
import socket
import traceback

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(port, out_q):
    try:
        import torch
        import torch.distributed as dist
        from helpers import int_bf16, to_dev_bf16
        from oracle import search_oracle as orc
        from denseretrievaltoolkits_amd import comm
        from denseretrievaltoolkits_amd import search as srch
        from denseretrievaltoolkits_amd.search import ShardedFlatIP
        from denseretrievaltoolkits_amd.trainer.losses import DistributedContrastiveLoss

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        assert dist.get_backend() == "nccl"
        comm.force_collectives(True)

        # count the collectives that reach torch.distributed with device tensors
        calls = {"all_gather_into_tensor": 0, "all_reduce": 0}
        real_ag, real_ar = dist.all_gather_into_tensor, dist.all_reduce

        def ag(out, src, *a, **kw):
            assert out.is_cuda and src.is_cuda
            calls["all_gather_into_tensor"] += 1
            return real_ag(out, src, *a, **kw)

        def ar(t, *a, **kw):
            assert t.is_cuda
            calls["all_reduce"] += 1
            return real_ar(t, *a, **kw)
        dist.all_gather_into_tensor, dist.all_reduce = ag, ar

        rng = np.random.default_rng(77)
        q = int_bf16(rng, (37, 768), -4, 4)
        p = int_bf16(rng, (120001, 768), -4, 4)
        k = 1000
        es, ei = orc.ip_topk(q, p, k)
        res = {}
        for proto in ("global_tau", "per_shard"):
            idx = ShardedFlatIP(768, device=dev, protocol=proto)
            idx.overlap_exchange = True   # the side-stream exchange through its own RCCL communicator
            idx.add_shard(to_dev_bf16(p, dev))
            assert idx._multi() and idx.offset == 0 and idx.ntotal == p.shape[0]
            qd = to_dev_bf16(q, dev)
            s, i = idx.search_device(qd, k)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(i.cpu().numpy(), ei)
            np.testing.assert_array_equal(s.cpu().numpy(), es)
            saved = srch.GROUP_QUERIES
            srch.GROUP_QUERIES = 16
            try:
                out = idx.search_batches([qd[a: a + 5] for a in range(0, q.shape[0], 5)], k)
                torch.cuda.synchronize()
            finally:
                srch.GROUP_QUERIES = saved
            np.testing.assert_array_equal(torch.cat([r[1] for r in out]).cpu().numpy(), ei)
            np.testing.assert_array_equal(torch.cat([r[0] for r in out]).cpu().numpy(), es)
            if proto == "global_tau":   # the groups' exchange ran on the side stream's own RCCL communicator
                assert idx._side_ch is not None and idx._side_ch.group is not None
            res[proto] = idx.fallbacks

        # comm helpers on device tensors
        t = torch.arange(12, dtype=torch.float32, device=dev).view(3, 4)
        st = comm.all_gather_stacked(t)
        assert st.shape == (1, 3, 4) and st.is_cuda and torch.equal(st[0], t)
        rows, sizes = comm.all_gather_rows(t)
        assert sizes == [3] and torch.equal(rows, t)
        m = comm.all_reduce_max_(t.clone())
        assert torch.equal(m, t)

        # DistributedContrastiveLoss through the RCCL all-gather: world 1 => the plain loss
        qr = torch.randn(4, 768, device=dev)
        pr = torch.randn(8, 768, device=dev)
        ld = DistributedContrastiveLoss()(qr, pr)
        tgt = torch.arange(4, device=dev) * 2
        lr = torch.nn.functional.cross_entropy(qr.double() @ pr.double().T, tgt)
        assert abs(ld.item() - lr.item()) <= 1e-4 * max(1.0, abs(lr.item())), (ld.item(), lr.item())
        res["calls"] = dict(calls)
        dist.destroy_process_group()
        out_q.put((True, res))
    except Exception:
        out_q.put((False, traceback.format_exc()))


def test_sharded_search_through_rccl_world1():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_worker, args=(_free_port(), q))
    pr.start()
    try:
        ok, res = q.get(timeout=240)
    finally:
        pr.join(timeout=60)
        if pr.is_alive():
            pr.kill()
    assert ok, res
    assert res["global_tau"] == 0, res
    # sample-list + packed-list gathers (global tau), (score, id, status) gathers (per shard),
    # offsets, helpers: dozens of device all-gathers went through RCCL
    assert res["calls"]["all_gather_into_tensor"] >= 10 and res["calls"]["all_reduce"] >= 1, res
