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
from ..evaluator.nq_eval import AnswerMatcher, has_answers
from ..search import ShardedFlatIP
from .losses import get_loss_function
from .scheduler import ConstantScheduler, CosineScheduler, InverseSquareRootScheduler, LinearScheduler

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
        sched = {"inverse": InverseSquareRootScheduler, "cosine": CosineScheduler, "linear": LinearScheduler,
                 "constant": ConstantScheduler}
        sname = getattr(a, "scheduler", None)
        if sname is not None and sname in sched:
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
        for batch in self.corpus_dataloader:
            data = {k: v.to(self.device) if v is not None else None for k, v in batch[1].items()}
            reps = self._encode(passage=data).p_reps
            if self.index is None:
                dim = reps.shape[1]
                self.index = ShardedFlatIP(dim, device=self.device)
            self.index.local.add(reps)
            ids_local.extend(list(batch[0]))
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

    def _search(self, q_reps: torch.Tensor, k: int) -> np.ndarray:
        """Global top-k ids for THIS rank's query batch (all ranks call it together).

        The reference searches each rank's own queries against a full host index on every
        rank (trainer.py:296-297).  Here the corpus is row-sharded, so the ranks' query
        batches (ragged: the last batch may differ per rank) are all-gathered, every rank
        scans its shard for all of them, and each keeps its own rows of the merged result."""
        if self.world == 1:
            _, i = self.index.search_device(q_reps, k)
            return i.cpu().numpy()
        allq, sizes = comm.all_gather_rows(q_reps.contiguous())
        _, ids = self.index.search_device(allq, k)
        lo = sum(sizes[: self.rank])
        return ids[lo: lo + sizes[self.rank]].cpu().numpy()

    def _doc_text(self, did_):
        t = self._doc_cache.get(did_)
        if t is None:
            t = self._doc_cache[did_] = self.corpus_dataloader.dataset[did_]["original"]
        return t

    def evaluate(self, query_loader, ep):
        self.model.eval()
        self._encoding_corpus(ep)
        self._index_corpus(ep)
        self._load_index(ep)
        a = self.training_args
        topk = a.topk if not isinstance(a.topk, str) else [int(x) for x in a.topk.split(",")]
        m_all = {f"{m}@{k}": 0.0 for m in ["MRR", "NDCG", "Recall"] for k in topk}
        eval_num = 0
        if self.world > 1 and hasattr(query_loader.sampler, "set_epoch"):
            query_loader.sampler.set_epoch(0)
        documents, queries, answers, qid, did = [], [], [], [], []
        k = a.retrieve_num
        matcher = AnswerMatcher()
        self._doc_cache = {}
        for batch in query_loader:
            data = {kk: v.to(self.device) if v is not None else None for kk, v in batch[1].items()}
            q_reps = self._encode(query=data).q_reps
            indices = self._search(q_reps, k)
            pos_index = np.zeros([len(indices), k], dtype=np.int8)
            docs, doc_ids = [], []
            for i, indice in enumerate(indices):
                eval_num += 1
                cols = np.flatnonzero(indice >= 0)
                doc_id = [self.idx[row] for row in indice[cols]]
                doc = [self._doc_text(did_) for did_ in doc_id]
                # has_answers over the whole list at once (nq_eval.AnswerMatcher: each passage
                # tokenised once per evaluation, not once per retrieving query)
                pos_index[i, cols] = matcher.match(doc_id, doc, batch[2][i])
                docs.append(doc)
                doc_ids.append(doc_id)
            documents.extend(docs)
            qid.extend(batch[0])
            answers.extend(batch[2])
            queries.extend(batch[3])
            did.extend(doc_ids)
            metrics = get_metrics(pos_index, topk)
            for key in m_all:
                m_all[key] += metrics[key]
        rdir = getattr(a, "retrieve_dir", "")
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
        for batch in pair_loader:
            data = {k: v.to(self.device) if v is not None else None for k, v in batch[1].items()}
            with torch.no_grad():
                scores = m(pos_pairs=data, neg_pairs=None).detach().cpu().numpy()
            for q, ans, d, s, did in zip(batch[0], batch[2], batch[3], scores, batch[4]):
                r = result.setdefault(q, ([], [], [], []))
                r[0].append(float(s[0]))
                r[1].append(int(matcher.match([did], [d], ans)[0]))
                r[2].append(d)
                r[3].append(did)
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
