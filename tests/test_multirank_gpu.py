"""GPU, several ranks: the distributed hot paths as real processes on the HIP kernels.

World 2 / 3 gloo process groups whose ranks share the one GPU of the test box
(collectives staged through host memory, comm.py; RCCL replaces gloo on a real
multi-GPU node, nothing else changes).  Every rank runs the real FlatIPIndex
scan kernels, the real packed / plain merges and the real encoder kernels:

* ShardedFlatIP, both protocols and the forced global-tau fallback, vs the
  oracle bit for bit; at world 3 against the reference's own top-k
  (tests/golden/corpus_topk.npz, merge_retrieval_results_by_score).
  Reference: trainer.py:220-262 (rank-0 index of every rank's rows),
  index.py:31-33 (search), utils.py:215-229 (partition merge).
* Trainer.evaluate at world 2 (query all-gather, object all-gather of doc ids,
  per-rank retrieve / metrics files) vs the oracle over the concatenated
  shard rows.  Reference: trainer.py:191-346.
* DRModel.forward and DistributedContrastiveLoss with negatives_x_device:
  the two ranks hold the two halves of the reference's golden batch
  (tests/golden/loss.npz), so loss = world x the golden loss and the local
  gradients = world x the golden gradient rows.  Reference:
  biencoder.py:103-119,243-254; losses.py:20-40.
* RRTrainer.evaluate at world 2: per-rank result files, rank-0 metrics ==
  the reference's file merge + argsort + get_metrics flow restated over the
  written files.  Reference: trainer.py:403-484.
"""
import json
import os
import socket
import traceback

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TIMEOUT = 240


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return torch.device("cuda", 0)


def _entry(fn, rank, world, port, out_q, args):
    import torch.distributed as dist
    try:
        dev = _init(rank, world, port)
        res = fn(rank, world, dev, *args)
        out_q.put((rank, True, res))
    except Exception:  # report, never hang the parent
        out_q.put((rank, False, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _spawn(fn, world, *args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, q, args)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, ok, v = q.get(timeout=TIMEOUT)
            res[r] = (ok, v)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    bad = {r: v for r, (ok, v) in res.items() if not ok}
    assert not bad, "\n".join(f"rank {r}:\n{v}" for r, v in bad.items())
    return {r: v for r, (_, v) in res.items()}


# ---------------------------------------------------------------------------
# sharded search
# ---------------------------------------------------------------------------
def _w_sharded(rank, world, dev, case):
    import torch
    from helpers import corpus_topk_golden, int_bf16, to_dev_bf16
    from oracle import search_oracle as orc
    from denseretrievaltoolkits_amd.search import ShardedFlatIP
    out = {}
    if case == "golden":
        q, p, k, _, gids, gscores = corpus_topk_golden()
        protocols = ["global_tau", "per_shard"]
    elif case == "gauss":
        # real-valued rows: the canonical exact-score order across shards (deltas all-reduced)
        from helpers import gauss_bf16
        rng = np.random.default_rng(43)
        q = gauss_bf16(rng, (37, 768))
        p = gauss_bf16(rng, (90001, 768))
        k = 1000
        protocols = ["global_tau"]
    elif case == "ties":
        # every row identical: all scores tie, far more than k candidates per shard pass tau,
        # so the global-tau lists overflow and the batch must take the per-shard fallback
        rng = np.random.default_rng(5)
        q = int_bf16(rng, (9, 256), -3, 3)
        p = np.repeat(int_bf16(rng, (1, 256), -3, 3), 50000, axis=0)
        k = 100
        protocols = ["global_tau"]
    else:
        rng = np.random.default_rng(41)
        q = int_bf16(rng, (37, 768), -4, 4)
        p = int_bf16(rng, (90001, 768), -4, 4)
        k = 1000
        protocols = ["global_tau", "per_shard"]
    es, ei = orc.ip_topk(q, p, k)
    lo, hi = orc.shard_bounds(p.shape[0], world, rank)
    for proto in protocols:
        idx = ShardedFlatIP(p.shape[1], device=dev, protocol=proto)
        idx.add_shard(to_dev_bf16(p[lo:hi], dev))
        assert idx.offset == lo and idx.ntotal == p.shape[0], (idx.offset, lo, idx.ntotal)
        s, i = idx.search_device(to_dev_bf16(q, dev), k)
        torch.cuda.synchronize()
        s, i = s.cpu().numpy(), i.cpu().numpy()
        np.testing.assert_array_equal(i, ei)
        if case == "gauss":   # exact sums rounded to fp32 (two fp64 orders: within one ulp)
            assert (np.abs(s.astype(np.float64) - es) <= np.spacing(np.abs(es))).all()
            assert idx.order_uncertified == 0
        else:
            np.testing.assert_array_equal(s, es)
        if case == "golden":
            np.testing.assert_array_equal(i, gids)
            np.testing.assert_array_equal(s, gscores)
        out[proto] = idx.fallbacks
        # batched search: ragged batches of 5 in groups of <= 16 queries (3 groups of up to 3 batches)
        # and with the shards' filter split into row chunks (every rank the same chunk count, the
        # gathered parts [world, chunks, ...] merged as one list set)
        from denseretrievaltoolkits_amd import search as srch
        saved = srch.GROUP_QUERIES, srch.GROUP_CHUNK_ROWS
        fb0 = idx.fallbacks
        for chunk_rows in ((saved[1], 20000) if case in ("int", "gauss") else (saved[1],)):
            srch.GROUP_QUERIES, srch.GROUP_CHUNK_ROWS = 16, chunk_rows
            try:
                if chunk_rows == 20000:
                    assert len(idx.group_chunks()) == -(-(-(-p.shape[0] // world)) // 20000)
                qd = to_dev_bf16(q, dev)
                res = idx.search_batches([qd[a: a + 5] for a in range(0, q.shape[0], 5)], k)
                torch.cuda.synchronize()
                if proto == "global_tau":
                    # round 6: the groups' exchange on a side stream + second communicator gives the same
                    # answer as the default one-stream form (redone batches not counted twice)
                    fb1 = idx.fallbacks
                    idx.overlap_exchange = True
                    res1 = idx.search_batches([qd[a: a + 5] for a in range(0, q.shape[0], 5)], k)
                    torch.cuda.synchronize()
                    idx.overlap_exchange = False
                    fb0 += idx.fallbacks - fb1
                    assert idx._side_ch is not None
                    for (s0, i0), (s1, i1) in zip(res, res1):
                        assert torch.equal(i0, i1) and torch.equal(s0, s1)
            finally:
                srch.GROUP_QUERIES, srch.GROUP_CHUNK_ROWS = saved
            np.testing.assert_array_equal(torch.cat([r[1] for r in res]).cpu().numpy(), ei)
            if case != "gauss":
                np.testing.assert_array_equal(torch.cat([r[0] for r in res]).cpu().numpy(), es)
        out[proto + "_batched"] = idx.fallbacks - fb0
        out[proto + "_order_uncertified"] = idx.order_uncertified
    return out


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_search_multiprocess_integer(world):
    res = _spawn(_w_sharded, world, "int")
    assert all(v["global_tau"] == 0 and v["global_tau_batched"] == 0 for v in res.values()), res


def test_sharded_search_multiprocess_reference_golden():
    """World 3 over the reference's golden corpus: ids and scores == merge_retrieval_results_by_score."""
    _spawn(_w_sharded, 3, "golden")


def test_sharded_search_multiprocess_gaussian_exact_order():
    """World 2 on Gaussian rows: ids == the fp64 oracle's bit for bit (canonical order, the
    exact-score deltas of the two shards summed by the all-reduce)."""
    res = _spawn(_w_sharded, 2, "gauss")
    assert all(v["global_tau"] == 0 and v["global_tau_batched"] == 0 for v in res.values()), res


def _w_sharded_large_k(rank, world, dev, data):
    """k > 2048 across ranks (round 6): each shard's canonical top-k with exact order keys, all-gathered
    and merged by exact key on the HIP kernels -- ids == the fp64 single-index order."""
    import torch
    from helpers import gauss_bf16, int_bf16, to_dev_bf16
    from oracle import search_oracle as orc
    from denseretrievaltoolkits_amd.search import ShardedFlatIP
    rng = np.random.default_rng(47)
    if data == "gauss":
        q = gauss_bf16(rng, (6, 768))
        p = gauss_bf16(rng, (150001, 768))   # shards of 75k rows > 65,536: the range-plan threshold
    else:
        q = int_bf16(rng, (5, 128), -2, 2)
        p = int_bf16(rng, (40000, 128), -2, 2)   # heavy exact ties, broken by global id
    k = 4096
    es, ei = orc.ip_topk(q, p, k)
    lo, hi = orc.shard_bounds(p.shape[0], world, rank)
    idx = ShardedFlatIP(p.shape[1], device=dev)
    idx.add_shard(to_dev_bf16(p[lo:hi], dev))
    s, i = idx.search_device(to_dev_bf16(q, dev), k)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(i.cpu().numpy(), ei)
    ulp = np.spacing(np.abs(es).astype(np.float32))
    assert (np.abs(s.cpu().numpy().astype(np.float64) - es) <= ulp).all()
    res = idx.search_batches([to_dev_bf16(q[:3], dev), to_dev_bf16(q[3:], dev)], k)
    np.testing.assert_array_equal(torch.cat([r[1] for r in res]).cpu().numpy(), ei)
    return True


@pytest.mark.parametrize("data", ["gauss", "int"])
def test_sharded_search_multiprocess_k_beyond_2048(data):
    _spawn(_w_sharded_large_k, 2, data)


def test_sharded_search_multiprocess_fallback():
    res = _spawn(_w_sharded, 2, "ties")
    # one batch of 9 queries; batched: batches of 5 + 4 in one group, both redone exactly -- round 6: the
    # redo merges every shard's exact keys, so no query is left in the fp32 order
    assert all(v["global_tau"] == 1 and v["global_tau_batched"] == 2 for v in res.values()), res
    assert all(v["global_tau_order_uncertified"] == 0 for v in res.values()), res


# ---------------------------------------------------------------------------
# Trainer.evaluate at world 2
# ---------------------------------------------------------------------------
WORDS = ["paris", "tower", "river", "york", "music", "rock", "roll", "river bank", "tokyo", "alps"]


def _w_trainer(rank, world, dev, tmp):
    from types import SimpleNamespace
    import torch
    from transformers import BertModel
    from oracle import bert_weights as bw
    from oracle import search_oracle as orc
    from denseretrievaltoolkits_amd import shards
    from denseretrievaltoolkits_amd.evaluator.metrics import get_metrics
    from denseretrievaltoolkits_amd.evaluator.nq_eval import has_answers
    from denseretrievaltoolkits_amd.model.biencoder import DRModel
    from denseretrievaltoolkits_amd.trainer.trainer import Trainer

    n_docs, n_q, k, bs = 2001, 41, 50, 128
    rng = np.random.default_rng(3)
    corpus = [{"original": " ".join(rng.choice(WORDS, size=int(rng.integers(3, 12))))} for _ in range(n_docs)]
    answers = [[str(rng.choice(WORDS))] for _ in range(n_q)]
    p_ids, p_mask = bw.token_batch(n_docs, 64, seed=11)
    q_ids, q_mask = bw.token_batch(n_q, 16, seed=12)
    # the reference's DistributedSampler(shuffle=False) split: pad to a multiple of world with
    # repeats, rank r takes indices r::world (corpus_dataloader.py:17-25); queries likewise but
    # left ragged here (the last rank has one query fewer) to exercise uneven batches
    pad = (-n_docs) % world
    order = list(range(n_docs)) + list(range(pad))
    mine = order[rank::world]
    qmine = list(range(n_q))[rank::world]

    class _L:
        def __init__(self, batches, dataset=None):
            self.batches, self.dataset, self.sampler = batches, dataset, None

        def __iter__(self):
            return iter(self.batches)

    def tb(a, idx):
        return torch.from_numpy(a[idx])

    cb = [(mine[a:a + bs], {"input_ids": tb(p_ids, mine[a:a + bs]), "attention_mask": tb(p_mask, mine[a:a + bs])})
          for a in range(0, len(mine), bs)]
    qb = [(qmine[a:a + 16], {"input_ids": tb(q_ids, qmine[a:a + 16]), "attention_mask": tb(q_mask, qmine[a:a + 16])},
           [answers[i] for i in qmine[a:a + 16]], [f"q{i}" for i in qmine[a:a + 16]])
          for a in range(0, len(qmine), 16)]
    torch.manual_seed(0)
    lm = BertModel(bw.bert_config(layers=1), add_pooling_layer=False).eval()
    bw.init_model_(lm, 5)
    model = DRModel(lm_q=lm, lm_p=lm, pooling="first", normalize=True)
    args = SimpleNamespace(loss_fn="SimpleContrastiveLoss", learning_rate=1e-5, optimizer="adamw", topk="1,5,20,50",
                           retrieve_num=k, retrieve_dir=os.path.join(tmp, "ret"), cache_train_dir=os.path.join(tmp, "cache"),
                           encode_corpus_dir=os.path.join(tmp, "emb"), index_order_dir=os.path.join(tmp, "idx"),
                           max_epochs=0, save_per_train=1, eval_per_train=1)
    tr = Trainer(args, model, corpus_dataloader=_L(cb, corpus), eval_loader=_L(qb))
    m = tr.evaluate(_L(qb), 0)
    assert m["query_num"] == len(qmine)

    # independent restatement: every rank's shard file in rank order = the global row order,
    # the gathered doc-id list maps rows to docs (trainer.py:307-308)
    rows = shards.load_rows(shards.list_shards(os.path.join(tmp, "emb"), 0), 0, len(order), "cpu").float().numpy()
    assert rows.shape == (len(order), 768)
    with open(os.path.join(tmp, "idx", "0.docid.txt"), encoding="utf-8") as f:
        row_doc = json.load(f)["id"]
    assert row_doc == [d for r in range(world) for d in order[r::world]]
    mod = tr.module
    with torch.no_grad():
        qr = torch.cat([mod(query={kk: v.to(dev) for kk, v in b[1].items()}).q_reps for b in qb]).float().cpu()
    q = qr.to(torch.bfloat16).float().numpy()
    es, ei = orc.ip_topk(q, rows, k)
    got = {}
    with open(os.path.join(tmp, "ret", f"0.{rank}.json"), encoding="utf-8") as f:
        for line in f:
            r = json.loads(line)
            got.setdefault(r["query_id"], []).append(r["doc_id"])
    first_row = {}
    for r_, d_ in enumerate(row_doc):
        first_row.setdefault(d_, r_)
    pos = np.zeros((len(qmine), k), np.int8)
    for qi, qid in enumerate(qmine):
        g = got[qid]
        assert len(g) == k
        for j in range(k):
            if g[j] != row_doc[ei[qi, j]]:
                # the GPU sums in fp32, the oracle in fp64: ids may differ only where the scores
                # agree within the north-star tolerance (1e-3)
                s_true = float(q[qi].astype(np.float64) @ rows[first_row[g[j]]].astype(np.float64))
                assert abs(s_true - es[qi, j]) <= 1e-3, (qid, j, g[j], s_true, es[qi, j])
            pos[qi, j] = has_answers(corpus[g[j]]["original"], answers[qid])
    # the reference accumulates get_metrics per query batch (trainer.py:319-321; NDCG is a
    # batch-level ratio, not a per-query sum) and divides by the query count
    ref = {}
    for a in range(0, len(qmine), 16):
        for key, v in get_metrics(pos[a:a + 16], [1, 5, 20, 50]).items():
            ref[key] = ref.get(key, 0.0) + v
    for key, v in ref.items():
        assert abs(m[key] - v / len(qmine)) < 1e-9, (key, m[key], v / len(qmine))
    with open(os.path.join(tmp, "cache", f"0.{rank}_metrics"), encoding="utf-8") as f:
        assert json.load(f)["query_num"] == len(qmine)
    return tr.index.fallbacks


def test_trainer_evaluate_world2(tmp_path):
    res = _spawn(_w_trainer, 2, str(tmp_path))
    assert set(res) == {0, 1}


# ---------------------------------------------------------------------------
# negatives_x_device: DRModel.forward / DistributedContrastiveLoss at world 2
# ---------------------------------------------------------------------------
def _w_xdev(rank, world, dev, golden_path):
    import torch
    from types import SimpleNamespace
    from transformers import BertModel
    from oracle import bert_weights as bw
    from denseretrievaltoolkits_amd.model.biencoder import DRModel
    from denseretrievaltoolkits_amd.trainer.losses import DistributedContrastiveLoss

    z = np.load(golden_path)
    q, p, n = z["n2_q"], z["n2_p"], int(z["n2_n"])
    bq = q.shape[0] // world
    ql = torch.from_numpy(q[rank * bq:(rank + 1) * bq]).to(dev).requires_grad_(True)
    pl = torch.from_numpy(p[rank * bq * n:(rank + 1) * bq * n]).to(dev).requires_grad_(True)
    loss = DistributedContrastiveLoss()(ql, pl)
    loss.backward()
    out = {}
    np.testing.assert_allclose(loss.item(), world * float(z["n2_loss"]), rtol=1e-5)
    np.testing.assert_allclose(ql.grad.cpu().numpy(), world * z["n2_dq"][rank * bq:(rank + 1) * bq], rtol=1e-4,
                               atol=1e-6)
    np.testing.assert_allclose(pl.grad.cpu().numpy(), world * z["n2_dp"][rank * bq * n:(rank + 1) * bq * n],
                               rtol=1e-4, atol=1e-6)

    # DRModel.forward with negatives_x_device on the HIP training tower (dropout off)
    cfg = bw.bert_config(layers=1)
    cfg.hidden_dropout_prob = 0.0
    cfg.attention_probs_dropout_prob = 0.0
    torch.manual_seed(0)
    lm = BertModel(cfg, add_pooling_layer=False)
    bw.init_model_(lm, 5)
    lm = lm.to(dev).train()
    model = DRModel(lm_q=lm, lm_p=lm, pooling="first", data_args=SimpleNamespace(train_n_passages=2),
                    train_args=SimpleNamespace(negatives_x_device=True)).train()
    qi, qm = bw.token_batch(3, 16, seed=100 + rank)
    pi, pm = bw.token_batch(6, 32, seed=200 + rank)
    o = model(query={"input_ids": torch.from_numpy(qi).to(dev), "attention_mask": torch.from_numpy(qm).to(dev)},
              passage={"input_ids": torch.from_numpy(pi).to(dev), "attention_mask": torch.from_numpy(pm).to(dev)})
    assert o.q_reps.shape == (3 * world, 768) and o.p_reps.shape == (6 * world, 768)
    o.q_reps.retain_grad()
    o.p_reps.retain_grad()
    o.loss.backward()
    qa = o.q_reps.detach().double().cpu()
    pa = o.p_reps.detach().double().cpu()
    qa.requires_grad_(True)
    pa.requires_grad_(True)
    tgt = torch.arange(qa.shape[0]) * 2
    ref = world * torch.nn.functional.cross_entropy(qa @ pa.T, tgt)
    ref.backward()
    np.testing.assert_allclose(o.loss.item(), ref.item(), rtol=1e-5)
    # fp32 softmax of scores in the hundreds vs fp64: absolute error relative to the largest entry
    for got_g, want_g in ((o.q_reps.grad, qa.grad), (o.p_reps.grad, pa.grad)):
        w = want_g.numpy()
        np.testing.assert_allclose(got_g.double().cpu().numpy(), w, rtol=1e-3, atol=2e-3 * np.abs(w).max())
    # the tower receives gradient only through its own (local) rows
    g = lm.embeddings.word_embeddings.weight.grad
    assert g is not None and torch.isfinite(g).all() and g.abs().sum() > 0
    out["loss"] = o.loss.item()
    return out


def test_negatives_x_device_world2():
    from conftest import REPO
    res = _spawn(_w_xdev, 2, os.path.join(REPO, "tests", "golden", "loss.npz"))
    # the x-device loss is the same global quantity on every rank
    assert abs(res[0]["loss"] - res[1]["loss"]) <= 1e-5 * abs(res[0]["loss"])


# ---------------------------------------------------------------------------
# RRTrainer.evaluate at world 2
# ---------------------------------------------------------------------------
def _w_rrtrainer(rank, world, dev, tmp):
    from types import SimpleNamespace
    import torch
    from transformers import BertModel
    from oracle import bert_weights as bw
    from denseretrievaltoolkits_amd.evaluator.metrics import get_metrics
    from denseretrievaltoolkits_amd.evaluator.nq_eval import has_answers
    from denseretrievaltoolkits_amd.model.linear import LinearHead
    from denseretrievaltoolkits_amd.model.reranker import RRModel
    from denseretrievaltoolkits_amd.trainer.trainer import RRTrainer

    n_q, per_q, L = 6, 20, 48
    rng = np.random.default_rng(9)
    docs = [" ".join(rng.choice(WORDS, size=int(rng.integers(2, 9)))) for _ in range(n_q * per_q)]
    answers = [[str(rng.choice(WORDS))] for _ in range(n_q)]
    ids, mask = bw.token_batch(n_q * per_q, L, seed=21)
    pairs = [(f"q{j // per_q}", j) for j in range(n_q * per_q)]
    mine = pairs[rank::world]                  # DistributedSampler(shuffle=False) split of the pairs
    batches = []
    for a in range(0, len(mine), 16):
        sel = [j for _, j in mine[a:a + 16]]
        batches.append(([q for q, _ in mine[a:a + 16]],
                         {"input_ids": torch.from_numpy(ids[sel]), "attention_mask": torch.from_numpy(mask[sel])},
                         [answers[j // per_q] for j in sel], [docs[j] for j in sel], [f"d{j}" for j in sel]))

    class _L:
        def __init__(self, b):
            self.b, self.sampler = b, None

        def __iter__(self):
            return iter(self.b)

    torch.manual_seed(0)
    lm = BertModel(bw.bert_config(layers=1), add_pooling_layer=False).eval()
    bw.init_model_(lm, 2)
    head = LinearHead(768, 1)
    with torch.no_grad():
        head.linear.weight.copy_(torch.from_numpy(bw.param_value(2, "rr_head.linear.weight", (1, 768))))
    model = RRModel(lm=lm, head=head, pooling="first")
    args = SimpleNamespace(loss_fn="none", learning_rate=1e-5, optimizer="adamw", topk=[1, 5, 10],
                           rr_result_dir=os.path.join(tmp, "rr"), cache_train_dir=os.path.join(tmp, "cache"))
    tr = RRTrainer(args, model)
    m = tr.evaluate(_L(batches), 3)
    import torch.distributed as dist
    dist.barrier()
    if rank != 0:
        assert m is None
        return None
    # the reference's rank-0 merge (trainer.py:449-482) restated over the per-rank files
    res = {}
    for fn in sorted(os.listdir(os.path.join(tmp, "rr"))):
        if fn.startswith("3."):
            with open(os.path.join(tmp, "rr", fn), encoding="utf-8") as f:
                for line in f:
                    dct = json.loads(line)
                    assert dct["match"] == int(has_answers(dct["document"], answers[int(dct["qid"][1:])]))
                    r = res.setdefault(dct["qid"], ([], []))
                    r[0].append(dct["score"])
                    r[1].append(dct["match"])
    assert len(res) == n_q and all(len(v[0]) == per_q for v in res.values())
    want = {f"{mt}@{k}": 0.0 for mt in ["MRR", "NDCG", "Recall"] for k in [1, 5, 10]}
    for _, (scores, is_true) in res.items():
        scores = np.array(scores)
        met = get_metrics([np.array(is_true)[np.argsort(-scores, kind="stable")]], [1, 5, 10])
        for key in want:
            want[key] += met[key]
    want["query_num"] = n_q
    for key in want:
        want[key] /= n_q           # the reference divides query_num too (trainer.py:476-478)
    for key, v in want.items():
        assert abs(m[key] - v) < 1e-12, (key, m[key], v)
    with open(os.path.join(tmp, "cache", "3.0_RR_metrics"), encoding="utf-8") as f:
        assert json.load(f) == pytest.approx(m)
    return {"n_q": len(res)}


def test_rrtrainer_evaluate_world2(tmp_path):
    res = _spawn(_w_rrtrainer, 2, str(tmp_path))
    assert res[1] is None and res[0] is not None


# ---------------------------------------------------------------------------
# Trainer.train_step under DDP (reference trainer.py:47-63,113-133; biencoder.py:103-119)
# ---------------------------------------------------------------------------
def _ddp_batch(rank, world, Bq, n, dev):
    import torch
    from oracle import bert_weights as bw
    q_ids, q_mask = bw.token_batch(world * Bq, 32, seed=21)
    p_ids, p_mask = bw.token_batch(world * Bq * n, 64, seed=22)
    if rank is not None:
        q_ids, q_mask = q_ids[rank * Bq:(rank + 1) * Bq], q_mask[rank * Bq:(rank + 1) * Bq]
        p_ids, p_mask = p_ids[rank * Bq * n:(rank + 1) * Bq * n], p_mask[rank * Bq * n:(rank + 1) * Bq * n]

    def t(x):
        return torch.from_numpy(x).to(dev)
    return ({"input_ids": t(q_ids), "attention_mask": t(q_mask)},
            {"input_ids": t(p_ids), "attention_mask": t(p_mask)})


def _ddp_model(dev, x_dev):
    from types import SimpleNamespace
    from transformers import BertModel
    from oracle import bert_weights as bw
    from denseretrievaltoolkits_amd.model.biencoder import DRModel
    lm = BertModel(bw.bert_config(layers=2), add_pooling_layer=False)   # dropout 0: deterministic
    bw.init_model_(lm, 7)
    return DRModel(lm_q=lm, lm_p=lm, pooling="first", data_args=SimpleNamespace(train_n_passages=2),
                   train_args=SimpleNamespace(negatives_x_device=x_dev))


def _w_ddp(rank, world, dev):
    import torch
    from types import SimpleNamespace
    from torch.nn.parallel import DistributedDataParallel as DDP
    from denseretrievaltoolkits_amd.trainer.trainer import Trainer
    Bq, n = 8, 2
    args = SimpleNamespace(loss_fn="SimpleContrastiveLoss", learning_rate=1e-5, optimizer="sgd")
    tr = Trainer(args, _ddp_model(dev, True))
    assert isinstance(tr.model, DDP)
    tr.model.train()
    loss = tr.train_step(list(_ddp_batch(rank, world, Bq, n, dev)))
    tr.optimizer.zero_grad()
    loss.backward()
    # DDP averaged the gradients over the ranks; every rank holds the same values
    got = {k: p.grad.detach().float().cpu() for k, p in tr.module.lm_q.named_parameters() if p.grad is not None}
    # one autograd node per layer: the tower's parameter gradients were released layer by layer
    names = set()

    def walk(fn, seen):
        if fn is None or fn in seen:
            return
        seen.add(fn)
        names.add(type(fn).__name__)
        for nxt, _ in fn.next_functions:
            walk(nxt, seen)
    walk(loss.grad_fn, set())
    out = {"loss": float(loss.detach()), "per_layer_nodes": sorted(x for x in names if "Fn" in x)}
    if rank == 0:
        # single process on the concatenated batch (in-batch negatives over all of it) = the
        # gradient DDP must reproduce: (1 / W) sum_r grad_r (W loss) with x-device gathering
        # (each rank's half encoded separately, as the ranks did: identical GEMM plans, so identical
        # bf16 reps; unnormalised BERT reps amplify any rounding difference into the scores)
        from denseretrievaltoolkits_amd.score_ce import score_ce
        ref_model = _ddp_model(dev, False).to(dev).train()
        halves = [_ddp_batch(r, world, Bq, n, dev) for r in range(world)]
        q = torch.cat([ref_model.encode_query(hq)[1] for hq, _ in halves])
        p = torch.cat([ref_model.encode_passage(hp)[1] for _, hp in halves])
        ref_loss, _ = score_ce(q, p, n, 1.0)
        ref_loss.backward()
        ref = {k: p.grad.detach().float().cpu() for k, p in ref_model.lm_q.named_parameters() if p.grad is not None}
        cos = {}
        for k, g in ref.items():
            a, b = got[k].reshape(-1).double(), g.reshape(-1).double()
            cos[k] = float((a @ b) / (a.norm() * b.norm() + 1e-30)) if b.norm() > 0 else float((a.norm() == 0))
        out.update(ref_loss=float(ref_loss.detach()), min_cos=min(cos.values()), worst=min(cos, key=cos.get),
                   n_params=len(ref), n_got=len(got))
    return out


def test_ddp_train_step_world2_matches_single_process():
    """Trainer wraps the model in DDP (find_unused_parameters=True, as the reference) at world 2;
    one train step with negatives_x_device on the HIP training tower: the loss equals the single-
    process loss on the concatenated batch (x W, the reference's scaling) and DDP's averaged
    parameter gradients equal that single process's gradients (cos >= 0.999 per tensor).  The single
    process encodes the two halves separately (the ranks' batch shapes) and scores their concatenation."""
    res = _spawn(_w_ddp, 2)
    r0 = res[0]
    assert abs(res[1]["loss"] - r0["loss"]) <= 1e-6 * max(1.0, abs(r0["loss"]))
    assert abs(r0["loss"] - 2 * r0["ref_loss"]) <= 1e-5 * abs(r0["ref_loss"]) + 1e-6, r0
    assert r0["n_got"] == r0["n_params"], r0
    assert r0["min_cos"] >= 0.999, r0
    assert "_LayerFnBackward" in r0["per_layer_nodes"] and "_EmbedFnBackward" in r0["per_layer_nodes"], r0
