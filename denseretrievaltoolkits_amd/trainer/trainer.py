"""Drop-in for DRT/trainer/trainer.py:Trainer on the MI355X hot path.

Same constructor, train / evaluate / save / load surface and output files
(retrieve/{ep}.{rank}.json, {ep}.{rank}_metrics, idx/{ep}.docid.txt).  The
corpus-encode -> index -> search pipeline is re-architected:

reference (trainer.py:191-346)                 this build
-----------------------------------------     ---------------------------------------------
encode on GPU, .cpu().numpy() per batch        encode on the HIP kernels; reps stay in HBM
np.save {ep}.{rank}.npy + JSON ids             rows appended to this rank's device shard
rank 0 loads every file into CPU faiss,        no file exchange: every rank keeps its shard;
writes the index; other ranks read it          doc ids all-gathered once (idx/{ep}.docid.txt)
each rank searches its own queries against     query reps all-gathered (RCCL), every rank
the FULL CPU index (faiss, OpenMP)             scans its shard, per-shard top-k all-gathered
                                               and merged on device; each rank keeps its rows

The reference's DistributedSampler corpus split (interleaved, padded with
repeats) is whatever the user's corpus_dataloader yields: rows map back to
doc ids through the gathered id list exactly as self.idx does at :307-308.
"""
from __future__ import annotations

import collections
import json
import logging
import os
from typing import List

import numpy as np
import torch
import torch.distributed as dist
from torch import optim
from torch.nn.parallel import DistributedDataParallel as DDP

from .. import comm
from ..evaluator.metrics import get_metrics
from ..evaluator.nq_eval import AnswerMatcher, DeviceRowMatcher, RowAnswerMatcher, has_answers
from ..search import ShardedFlatIP, _stage_host
from .losses import get_loss_function

logger = logging.getLogger(__name__)


def _world():
    return (dist.get_world_size(), dist.get_rank()) if dist.is_initialized() else (1, 0)


class Trainer:
    def __init__(self, training_args, model, corpus_dataloader=None, train_loader=None, eval_loader=None,
                 test_loader=None):
        self.training_args = training_args
        self.model = model
        self._wrapper_model()
        self.loss_fn = get_loss_function(training_args)
        self.train_loader = train_loader
        self._get_optimizer_and_scheduler()
        self.corpus_dataloader = corpus_dataloader
        self.eval_loader = eval_loader
        self.test_loader = test_loader
        self.start_epoch = 0
        self.eval_method = getattr(training_args, "eval_method", "metrics")
        self.index = None
        self.idx: List = []
        if eval_loader is not None and isinstance(training_args.topk, str):
            training_args.topk = [int(k) for k in training_args.topk.split(",")]

    # ------------------------------------------------------------------
    def _wrapper_model(self):
        self.world, self.rank = _world()
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        # one process per GPU (run.sh: torch.distributed.launch); ranks beyond the visible
        # devices share them (the multi-rank tests run several gloo ranks on one GPU)
        dev_index = self.local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev_index)
        self.device = torch.device("cuda", dev_index)
        if dist.is_initialized():
            dist.barrier()
        self.model = self.model.to(self.device)
        if self.world > 1:
            self.model = DDP(self.model, device_ids=[dev_index], output_device=dev_index,
                             find_unused_parameters=True)

    @property
    def module(self):
        return self.model.module if isinstance(self.model, DDP) else self.model

    def _get_optimizer_and_scheduler(self):
        a = self.training_args
        params = [p for p in self.model.parameters() if p.requires_grad]
        kw = {"lr": a.learning_rate}
        kw.update(getattr(a, "optimizer_kwargs", {}) or {})
        classes = collections.defaultdict(lambda: optim.AdamW, {
            "adam": optim.Adam, "adamw": optim.AdamW, "sgd": optim.SGD, "adagrad": optim.Adagrad,
            "rmsprop": optim.RMSprop})
        name = getattr(a, "optimizer", "adam")
        if name == "adafactor":
            import transformers
            kw.update(getattr(a, "adafactor_kwargs", {}) or {})
            opt = transformers.Adafactor(params=params, **kw)
        else:
            opt = classes[name](params=params, **kw)
        sname = getattr(a, "scheduler", None)
        if sname is not None and sname in ("inverse", "cosine", "linear", "constant"):
            # the LR schedulers are off the hot path (scalar lr arithmetic): the user's own
            # DRT.trainer.scheduler classes wrap the optimizer, as the reference does (trainer.py:85-112)
            import importlib
            try:
                us = importlib.import_module("DRT.trainer.scheduler")
            except ImportError as e:
                raise ImportError(
                    f"scheduler={sname!r} uses the reference's own LR schedulers (DRT.trainer.scheduler), which "
                    "are not part of this package: put the DRT checkout on PYTHONPATH (INTEGRATION.md) or pass "
                    "scheduler=None") from e
            sched = {"inverse": us.InverseSquareRootScheduler, "cosine": us.CosineScheduler,
                     "linear": us.LinearScheduler, "constant": us.ConstantScheduler}
            skw = dict(getattr(a, "scheduler_kwargs", {}) or {})
            skw.setdefault("max_lr", a.learning_rate)
            opt = sched[sname](base_optimizer=opt, **skw)
        self.optimizer = opt

    # ------------------------------------------------------------------
    def train_step(self, inputs):
        encoded = self.model(query=inputs[0], passage=inputs[1])
        return encoded.loss

    def train(self):
        self.model.train()
        for ep in range(self.start_epoch, self.training_args.max_epochs):
            if self.world > 1 and hasattr(self.train_loader.sampler, "set_epoch"):
                self.train_loader.sampler.set_epoch(ep)
            for batch in self.train_loader:
                prepared = [{k: v.to(self.device) if v is not None else None for k, v in data.items()}
                            for data in batch]
                loss = self.train_step(prepared)
                self.optimizer.zero_grad()
                loss.backward()
                self.optimizer.step()
            if dist.is_initialized():
                dist.barrier()
            if (ep + 1) % self.training_args.save_per_train == 0:
                self.save(ep + 1)
            if (ep + 1) % self.training_args.eval_per_train == 0:
                self.evaluate(self.eval_loader, ep + 1)
                self.model.train()
        self.evaluate(self.test_loader, -1)

    # ------------------------------------------------------------------
    def _encode(self, query=None, passage=None):
        m = self.module
        with torch.no_grad():
            out = m(query=query, passage=passage)
        return out

    def _encoding_corpus(self, ep):
        """Encode this rank's corpus batches straight into its device shard."""
        dim = None
        ids_local: List = []
        self.index = None
        # answers of evaluate are matched against the passages' tokens: the passages of this
        # rank's shard are tokenised here, on the host, while the GPU encodes the next batches
        ds = getattr(self.corpus_dataloader, "dataset", None)
        self._matcher = RowAnswerMatcher(0) if (self.prefill_answer_tokens and ds is not None) else None
        prefill = self._matcher is not None
        for batch in self.corpus_dataloader:
            data = {k: self._to_device(v) for k, v in batch[1].items()}
            reps = self._encode(passage=data).p_reps
            if self.index is None:
                dim = reps.shape[1]
                self.index = ShardedFlatIP(dim, device=self.device)
                try:   # one allocation for the whole shard when the loader knows its length
                    self.index.local.reserve(len(self.corpus_dataloader) * reps.shape[0])
                except TypeError:
                    pass
            row0 = self.index.local.ntotal
            self.index.local.add(reps)
            ids_local.extend(list(batch[0]))
            if self._matcher is not None:
                dids = list(batch[0])
                self._matcher.ensure_rows(row0 + len(dids))
                if prefill:
                    try:
                        self._matcher.fill(np.arange(row0, row0 + len(dids)),
                                           lambda r, _d=dids, _o=row0: ds[_d[r - _o]]["original"])
                    except (KeyError, TypeError, IndexError):
                        self._matcher = None   # no 'original' texts here: matched on demand in evaluate
                        continue
                    # bounded: past the budget the remaining rows are tokenised only if a query
                    # retrieves them (the matcher's slots grow with the rows actually tokenised)
                    prefill = self._matcher.token_bytes < self.prefill_answer_max_bytes
        if self.index is None:
            raise ValueError("empty corpus")
        self._ids_local = ids_local
        d = getattr(self.training_args, "encode_corpus_dir", "")
        if d:
            os.makedirs(d, exist_ok=True)
            self.index.save_shard(d, ep)   # {ep}.{rank}.bf16.npy, memory-mappable (shards.py)
            with open(os.path.join(d, f"{ep}.{self.rank}.json"), "w", encoding="utf-8") as f:
                json.dump({"id": ids_local}, f, ensure_ascii=False)
        if dist.is_initialized():
            dist.barrier()

    def _index_corpus(self, ep):
        """Agree on global row ids (shard offsets) and the row -> doc-id map."""
        self.index.sync_offsets()
        if getattr(self, "_matcher", None) is not None and self.world > 1:
            self._matcher.rebase(self.index.offset, self.index.local.ntotal, self.index.ntotal)
        if self.world > 1:
            gathered = [None] * self.world
            dist.all_gather_object(gathered, self._ids_local)
            self.idx = [x for part in gathered for x in part]
        else:
            self.idx = list(self._ids_local)
        d = getattr(self.training_args, "index_order_dir", "")
        if d and self.rank == 0:
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, f"{ep}.docid.txt"), "w", encoding="utf-8") as f:
                json.dump({"id": self.idx}, f, ensure_ascii=False)

    def _load_index(self, ep):
        if dist.is_initialized():
            dist.barrier()

    # ------------------------------------------------------------------
    # evaluate: query encode + search + answer matching, pipelined (reference trainer.py:269-346)
    # ------------------------------------------------------------------
    # Query batches are encoded in windows of up to ENCODE_WINDOW queries of one sequence length
    # (one tower pass over thousands of queries runs the large-GEMM plans instead of a 128-query
    # pass per loader batch), then searched in batches of SEARCH_BATCH through the certified,
    # pipelined product path (search.FlatIPIndex / ShardedFlatIP.search_batches_iter): batch j + 1
    # is on the GPU while the host matches answers for batch j, whose ids land in pinned memory
    # behind an event.  Metrics stay per LOADER batch (get_metrics' NDCG is a batch-level ratio).
    ENCODE_WINDOW = 4096
    SEARCH_BATCH = 128
    # one rank: a whole window's searches are enqueued before the next window's tower pass, so the host
    # certifies and matches the window while the GPU runs that pass (in-process A/B, tools/c2_ab.py,
    # profiles/r04ab_c2_window_order_ab.log: query stage 0.150 / 0.152 s vs 0.191 / 0.211 s with the
    # next tower pass queued behind the window's first searches)
    EAGER_WINDOW_SEARCH = True
    prefill_answer_tokens = True
    # host (and, mirrored, HBM) bytes of passage tokens prefilled during the corpus encode
    prefill_answer_max_bytes = 1 << 30

    def _to_device(self, v):
        if v is None or not isinstance(v, torch.Tensor):
            return v
        if v.is_cuda:
            return v
        return v.pin_memory().to(self.device, non_blocking=True)

    def _query_windows(self, query_loader):
        """Yields lists of loader batches (inputs on the device) of one sequence length, up to
        ENCODE_WINDOW queries each."""
        win, n, L = [], 0, None
        for batch in query_loader:
            data = {kk: self._to_device(v) for kk, v in batch[1].items()}
            bl = data["input_ids"].shape[1]
            nb = data["input_ids"].shape[0]
            if win and (bl != L or n + nb > self.ENCODE_WINDOW):
                yield win
                win, n = [], 0
            win.append((batch, data))
            n += nb
            L = bl
        if win:
            yield win

    def _encode_window(self, win) -> torch.Tensor:
        datas = [d for _, d in win]
        if len(datas) == 1:
            data = datas[0]
        else:
            data = {kk: (torch.cat([d[kk] for d in datas]) if datas[0][kk] is not None else None) for kk in datas[0]}
        return self._encode(query=data).q_reps

    def _search_rows(self, q_reps: torch.Tensor, k: int, to_host: bool = True):
        """Yields (row0, ids [n, k] host) for consecutive row ranges of this rank's query reps.

        W = 1: the window's rows in SEARCH_BATCH batches.  W > 1: the corpus is row-sharded, so the
        ranks' windows (ragged: a rank may have fewer or no queries left) are all-gathered, every
        rank scans its shard for all of them (grouped global-threshold protocol), and each keeps
        its own rows of the merged result (the reference searches each rank's own queries against
        a full host index on every rank, trainer.py:296-297)."""
        sb = self.SEARCH_BATCH
        if self.world == 1:
            batches = [q_reps[a: a + sb] for a in range(0, q_reps.shape[0], sb)]
            for j, (_, ids) in enumerate(self.index.local.search_batches_iter(batches, k, to_host=to_host)):
                yield j * sb, ids
            return
        # every rank hands the collective the same dtype (a rank with no queries left sends an
        # empty fp32 tensor)
        allq, sizes = comm.all_gather_rows(q_reps.float().contiguous())
        lo = sum(sizes[: self.rank])
        hi = lo + sizes[self.rank]
        batches = [allq[a: a + sb] for a in range(0, allq.shape[0], sb)]
        for j, (_, ids) in enumerate(self.index.search_batches_iter(batches, k, to_host=to_host)):
            a, b = max(lo, j * sb), min(hi, (j + 1) * sb)
            if a < b:
                yield a - lo, ids[a - j * sb: b - j * sb]

    def _search(self, q_reps: torch.Tensor, k: int) -> np.ndarray:
        """Global top-k ids [n, k] (host) of THIS rank's query reps (all ranks call it together)."""
        out = np.empty((q_reps.shape[0], k), dtype=np.int64)
        for row0, ids in self._search_rows(q_reps, k):
            out[row0: row0 + ids.shape[0]] = ids
        return out

    def _eval_results(self, query_loader, k: int, to_host: bool = True):
        """Yields (loader batch, ids [B, k]) in loader order (all ranks call it together); the ids are
        host arrays, or device tensors with ``to_host`` False (the device answer matcher's input)."""
        windows = self._query_windows(query_loader)
        d = self.index.d

        def encode_next():
            w = next(windows, None)
            return w, (self._encode_window(w) if w is not None else None)

        nxt = encode_next()
        while True:
            win, q_reps = nxt
            nxt = None
            if self.world > 1:
                # every rank takes part in every window's collectives until all are exhausted
                n_local = 0 if win is None else sum(dd["input_ids"].shape[0] for _, dd in win)
                if sum(comm.all_gather_sizes(n_local, self.device)) == 0:
                    return
            elif win is None:
                return
            if win is None:
                q_reps = torch.empty((0, d), dtype=torch.float32, device=self.device)
                win = []
            n = q_reps.shape[0]
            ids_all = np.empty((n, k), dtype=np.int64) if to_host else \
                torch.empty((n, k), dtype=torch.int64, device=self.device)
            done, bi, b0 = 0, 0, 0
            if self.world == 1 and self.EAGER_WINDOW_SEARCH and n:
                # the whole window's searches first, then the next window's tower pass
                sb = self.SEARCH_BATCH
                loc = self.index.local
                pend = loc.enqueue_batches([q_reps[a: a + sb] for a in range(0, n, sb)], k, to_host=to_host)
                nxt = encode_next()
                rows_iter = ((j * sb, loc.finish_batch(p_)[1]) for j, p_ in enumerate(pend))
            else:
                rows_iter = self._search_rows(q_reps, k, to_host)
            for row0, ids in rows_iter:
                if nxt is None:
                    # the next window's tower pass goes on the GPU behind this window's first search
                    # runs, so it runs while the host matches this window's batches
                    nxt = encode_next()
                ids_all[row0: row0 + ids.shape[0]] = ids
                done = row0 + ids.shape[0]
                # hand out every loader batch whose rows are complete (host work overlaps the
                # GPU's next search batch)
                while bi < len(win) and b0 + win[bi][1]["input_ids"].shape[0] <= done:
                    nb = win[bi][1]["input_ids"].shape[0]
                    yield win[bi][0], ids_all[b0: b0 + nb]
                    b0 += nb
                    bi += 1
            while bi < len(win):
                nb = win[bi][1]["input_ids"].shape[0]
                yield win[bi][0], ids_all[b0: b0 + nb]
                b0 += nb
                bi += 1
            if nxt is None:
                nxt = encode_next()

    def _doc_text(self, did_):
        t = self._doc_cache.get(did_)
        if t is None:
            t = self._doc_cache[did_] = self.corpus_dataloader.dataset[did_]["original"]
        return t

    # stage timing of evaluate (bench.py's evaluate_c2 leg): synchronises the device once between
    # the corpus stage and the query stage when on; off by default
    profile_eval = False

    def evaluate(self, query_loader, ep):
        import time
        t0 = time.perf_counter()
        self.model.eval()
        self._encoding_corpus(ep)
        self._index_corpus(ep)
        self._load_index(ep)
        if self.profile_eval:
            torch.cuda.synchronize(self.device)
        t1 = time.perf_counter()
        t_host = 0.0
        a = self.training_args
        topk = a.topk if not isinstance(a.topk, str) else [int(x) for x in a.topk.split(",")]
        m_all = {f"{m}@{k}": 0.0 for m in ["MRR", "NDCG", "Recall"] for k in topk}
        eval_num = 0
        if self.world > 1 and hasattr(query_loader.sampler, "set_epoch"):
            query_loader.sampler.set_epoch(0)
        documents, queries, answers, qid, did = [], [], [], [], []
        k = a.retrieve_num
        rdir = getattr(a, "retrieve_dir", "")
        self._doc_cache = {}
        # vectorised has_answers over each batch's retrieved rows (nq_eval.RowAnswerMatcher: every
        # passage tokenised once per evaluation -- this rank's shard already during the corpus encode)
        matcher = getattr(self, "_matcher", None)
        if matcher is None:
            matcher = RowAnswerMatcher(len(self.idx))
        matcher.ensure_rows(len(self.idx))
        if self.device.type == "cuda":   # the token matrix in HBM: rows gathered / compared on the GPU
            matcher = DeviceRowMatcher(matcher, self.device)

        def text_of(row):
            return self._doc_text(self.idx[row])

        # device metrics: the matches and get_metrics of every loader batch stay on the GPU (summed there,
        # read back once after the last batch) and the search's ids never leave the device -- unless the
        # retrieve/ output file needs the documents on the host.  (A batch beyond the metrics kernel's limits
        # -- k > 2048 on the large-k search path, > 4096 queries, > 16 cut-offs -- has its get_metrics taken
        # on the host inside match_metrics, into the same sums.)
        dev_metrics = isinstance(matcher, DeviceRowMatcher) and not rdir
        if dev_metrics:
            macc = torch.zeros(3 * len(topk), dtype=torch.float64, device=self.device)
            topk_dev = torch.tensor(topk, dtype=torch.int32, device=self.device)

        def finish(pend):
            # batch j's matches are read (and its metrics taken) after batch j + 1's are enqueued
            batch, indices, match = pend
            pos_index = match.get()
            if rdir:   # the retrieved documents are only needed for the retrieve/ output file
                for indice in indices:
                    doc_id = [self.idx[row] for row in indice[indice >= 0]]
                    documents.append([self._doc_text(did_) for did_ in doc_id])
                    did.append(doc_id)
            qid.extend(batch[0])
            answers.extend(batch[2])
            queries.extend(batch[3])
            metrics = get_metrics(pos_index, topk)
            for key in m_all:
                m_all[key] += metrics[key]

        pend = None
        tw = {"results_wait_s": 0.0, "match_issue_s": 0.0, "match_finish_s": 0.0}
        res_iter = self._eval_results(query_loader, k, to_host=not dev_metrics)
        while True:
            t0w = time.perf_counter()
            nxt_res = next(res_iter, None)
            tw["results_wait_s"] += time.perf_counter() - t0w
            if nxt_res is None:
                break
            batch, indices = nxt_res
            th = time.perf_counter()
            if dev_metrics:
                matcher.match_metrics(indices, text_of, batch[2], topk_dev, macc)
                eval_num += len(indices)
                t_host += time.perf_counter() - th
                tw["match_issue_s"] += time.perf_counter() - th
                continue
            if hasattr(matcher, "match_rows_async"):
                cur = (batch, indices, matcher.match_rows_async(indices, text_of, batch[2]))
            else:
                cur = (batch, indices, _Ready(matcher.match_rows(indices, text_of, batch[2])))
            eval_num += len(indices)
            tm = time.perf_counter()
            tw["match_issue_s"] += tm - th
            if pend is not None:
                finish(pend)
            pend = cur
            tw["match_finish_s"] += time.perf_counter() - tm
            t_host += time.perf_counter() - th
        if pend is not None:
            th = time.perf_counter()
            finish(pend)
            t_host += time.perf_counter() - th
        if dev_metrics:
            torch.cuda.current_stream(self.device).wait_stream(matcher.stream)
            acc = macc.cpu().numpy()
            T = len(topk)
            for t, kk in enumerate(topk):
                m_all[f"Recall@{kk}"] += float(acc[t])
                m_all[f"MRR@{kk}"] += float(acc[T + t])
                m_all[f"NDCG@{kk}"] += float(acc[2 * T + t])
        t2 = time.perf_counter()
        if rdir:
            os.makedirs(rdir, exist_ok=True)
            with open(os.path.join(rdir, f"{ep}.{self.local_rank}.json"), "w", encoding="utf-8") as f:
                for i in range(len(did)):
                    for doc, d in zip(documents[i], did[i]):
                        json.dump({"doc_id": d, "query_id": qid[i], "query": queries[i], "document": doc,
                                   "answers": answers[i]}, f, ensure_ascii=False)
                        f.write("\n")
        for key in m_all:
            m_all[key] = m_all[key] / max(eval_num, 1)
            logger.info("%s %s", key, m_all[key])
        m_all["query_num"] = eval_num
        cdir = getattr(a, "cache_train_dir", "")
        if cdir:
            os.makedirs(cdir, exist_ok=True)
            with open(os.path.join(cdir, f"{ep}.{self.local_rank}_metrics"), "w", encoding="utf-8") as f:
                json.dump(m_all, f, ensure_ascii=False)
        if dist.is_initialized():
            dist.barrier()
        self.last_metrics = m_all
        self.last_eval_timing = {"corpus_s": t1 - t0, "queries_s": t2 - t1, "host_match_s": t_host,
                                 "files_s": time.perf_counter() - t2, **tw}
        return m_all

    # ------------------------------------------------------------------
    def save(self, i_epoch):
        if self.rank == 0:
            path = os.path.join(self.training_args.cache_train_dir, "result" + str(i_epoch))
            os.makedirs(path, exist_ok=True)
            self.module.save(path)

    def _get_checkpoint(self, i_epoch):
        return {"state_dict": self.module.get_model_ckpt(), "optimizer": self.optimizer.state_dict(),
                "epoch": i_epoch}

    def load(self, filename, ckpt_type=None):
        checkpoint = torch.load(filename, map_location=self.device, weights_only=True)
        if ckpt_type is None:
            self.start_epoch = checkpoint["epoch"] + 1
            self.module.load(checkpoint["state_dict"])
            self.optimizer.load_state_dict(checkpoint["optimizer"])


class _Ready:
    """An already computed match result with the pending-match interface."""
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v

    def get(self):
        return self.v


class RRTrainer(Trainer):
    """Drop-in for RRTrainer (DRT/trainer/trainer.py:392-484): pair scores on the HIP
    reranker; per-rank result files as the reference, merged on rank 0 through an
    object all-gather instead of re-reading every rank's file."""

    def train_step(self, inputs):
        return self.model(pos_pairs=inputs[0], neg_pairs=inputs[1]).loss

    def evaluate(self, pair_loader, ep):
        self.model.eval()
        a = self.training_args
        topk = a.topk if not isinstance(a.topk, str) else [int(x) for x in a.topk.split(",")]
        if self.world > 1 and hasattr(pair_loader.sampler, "set_epoch"):
            pair_loader.sampler.set_epoch(0)
        result = {}
        m = self.module
        matcher = AnswerMatcher()

        def finish(pend):
            # host work of a batch whose scores were staged behind an event: runs while the GPU
            # scores the next batch (the reference copies each batch's scores back synchronously)
            batch, (hs,), ev = pend
            ev.synchronize()
            scores = hs.numpy()
            for q, ans, d, sc, did in zip(batch[0], batch[2], batch[3], scores, batch[4]):
                r = result.setdefault(q, ([], [], [], []))
                r[0].append(float(sc[0]))
                r[1].append(int(matcher.match([did], [d], ans)[0]))
                r[2].append(d)
                r[3].append(did)

        pend = None
        for batch in pair_loader:
            data = {k: self._to_device(v) for k, v in batch[1].items()}
            with torch.no_grad():
                scores = m(pos_pairs=data, neg_pairs=None).detach()
            cur = (batch,) + _stage_host(scores.float())
            if pend is not None:
                finish(pend)
            pend = cur
        if pend is not None:
            finish(pend)
        rdir = getattr(a, "rr_result_dir", "")
        if rdir:
            os.makedirs(rdir, exist_ok=True)
            with open(os.path.join(rdir, f"{ep}.{self.local_rank}.json"), "w", encoding="utf-8") as f:
                for qid, (scs, js, ds, dids) in result.items():
                    for s, j, d, did in zip(scs, js, ds, dids):
                        json.dump({"qid": qid, "did": did, "score": s, "match": j, "document": d}, f,
                                  ensure_ascii=False)
                        f.write("\n")
        local = {q: (r[0], r[1]) for q, r in result.items()}
        if self.world > 1:
            parts = [None] * self.world
            dist.all_gather_object(parts, local)
        else:
            parts = [local]
        m_all = None
        if self.rank == 0:
            merged = {}
            for part in parts:
                for q, (scs, js) in part.items():
                    mm = merged.setdefault(q, ([], []))
                    mm[0].extend(scs)
                    mm[1].extend(js)
            m_all = {f"{mt}@{k}": 0.0 for mt in ["MRR", "NDCG", "Recall"] for k in topk}
            n = 0
            for q, (scs, js) in merged.items():
                n += 1
                order = np.argsort(-np.asarray(scs), kind="stable")
                metrics = get_metrics([np.asarray(js)[order]], topk)
                for key in m_all:
                    m_all[key] += metrics[key]
            m_all["query_num"] = n
            for key in m_all:
                m_all[key] = m_all[key] / max(n, 1)
            cdir = getattr(a, "cache_train_dir", "")
            if cdir:
                os.makedirs(cdir, exist_ok=True)
                with open(os.path.join(cdir, f"{ep}.{self.local_rank}_RR_metrics"), "w", encoding="utf-8") as f:
                    json.dump(m_all, f, ensure_ascii=False)
        if dist.is_initialized():
            dist.barrier()
        self.last_metrics = m_all
        return m_all
