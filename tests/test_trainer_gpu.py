"""GPU: Trainer.evaluate end to end on world size 1.

Corpus encode on the HIP encoder -> rows appended to the HBM shard -> shard file
({ep}.{rank}.bf16.npy) -> query encode -> HIP top-k -> doc-id map -> vectorised
answer matching -> get_metrics, and the reference's output files
(DRT/trainer/trainer.py:191-346).  Checked against an independent restatement:
the shard file's rows searched by the CPU oracle, answers matched by the
has_answers restatement (pinned to the reference by tests/golden/answers.json),
metrics by the get_metrics restatement (pinned by tests/golden/metrics.json).
"""
import json
import os
from types import SimpleNamespace

import numpy as np
import pytest

from oracle import bert_weights as bw
from oracle import search_oracle as orc

pytestmark = pytest.mark.gpu

WORDS = ["paris", "tower", "river", "york", "music", "rock", "roll", "river bank", "tokyo", "alps"]


def _loaders(n_docs, n_q, L_p, L_q, bs):
    import torch
    rng = np.random.default_rng(3)
    corpus = [{"original": " ".join(rng.choice(WORDS, size=int(rng.integers(3, 12))))} for _ in range(n_docs)]
    p_ids, p_mask = bw.token_batch(n_docs, L_p, seed=11)
    q_ids, q_mask = bw.token_batch(n_q, L_q, seed=12)

    ds = list(corpus)
    cbatches = [(list(range(a, min(n_docs, a + bs))),
                 {"input_ids": torch.from_numpy(p_ids[a:a + bs]), "attention_mask": torch.from_numpy(p_mask[a:a + bs])})
                for a in range(0, n_docs, bs)]
    answers = [[str(rng.choice(WORDS))] for _ in range(n_q)]
    qbatches = [(list(range(a, min(n_q, a + bs))),
                 {"input_ids": torch.from_numpy(q_ids[a:a + bs]), "attention_mask": torch.from_numpy(q_mask[a:a + bs])},
                 answers[a:a + bs], [f"q{i}" for i in range(a, min(n_q, a + bs))])
                for a in range(0, n_q, bs)]

    class _L:
        def __init__(self, batches, dataset=None):
            self.batches, self.dataset, self.sampler = batches, dataset, None

        def __iter__(self):
            return iter(self.batches)

    return _L(cbatches, ds), _L(qbatches), corpus, answers


@pytest.mark.parametrize("layers,n_docs,n_q,k,L_p,L_q,bs,files", [
    (1, 3000, 40, 50, 64, 16, 256, True),
    # no retrieve/ file: matches and metrics stay on the device (drt_hit_metrics_i8), ids never leave it
    (1, 3000, 40, 50, 64, 16, 256, False),
    # BASELINE config C1's shape (1k passages / 32 queries, BERT-base) at k = 1000 = every row
    (12, 1000, 32, 1000, 128, 32, 128, True),
    (12, 1000, 32, 1000, 128, 32, 128, False),
    # retrieve_num beyond the candidate-list kernels (the large-k search path) and beyond the device
    # metrics kernel's k <= 2048: that batch's get_metrics runs on the host, into the same sums
    (1, 5000, 24, 3000, 64, 16, 256, False),
    (1, 5000, 24, 3000, 64, 16, 256, True),
])
def test_evaluate_end_to_end_matches_oracle(dev, tmp_path, layers, n_docs, n_q, k, L_p, L_q, bs, files):
    import torch
    from transformers import BertModel
    from denseretrievaltoolkits_amd import shards
    from denseretrievaltoolkits_amd.evaluator.metrics import get_metrics
    from denseretrievaltoolkits_amd.evaluator.nq_eval import has_answers
    from denseretrievaltoolkits_amd.model.biencoder import DRModel
    from denseretrievaltoolkits_amd.trainer.trainer import Trainer

    torch.manual_seed(0)
    lm = BertModel(bw.bert_config(layers=layers), add_pooling_layer=False).eval()
    bw.init_model_(lm, 5)
    model = DRModel(lm_q=lm, lm_p=lm, pooling="first", normalize=True)
    cl, ql, corpus, answers = _loaders(n_docs, n_q, L_p, L_q, bs)
    topk = [1, 5, 20, k]
    args = SimpleNamespace(loss_fn="SimpleContrastiveLoss", learning_rate=1e-5, optimizer="adamw",
                           topk=",".join(map(str, topk)),
                           retrieve_num=k, retrieve_dir=str(tmp_path / "ret") if files else "",
                           cache_train_dir=str(tmp_path / "cache"),
                           encode_corpus_dir=str(tmp_path / "emb"), index_order_dir=str(tmp_path / "idx"),
                           max_epochs=0, save_per_train=1, eval_per_train=1)
    tr = Trainer(args, model, corpus_dataloader=cl, eval_loader=ql)
    m = tr.evaluate(ql, 0)
    assert m["query_num"] == n_q

    # independent restatement from the written shard file + a fresh query encode
    rows = shards.load_rows(shards.list_shards(str(tmp_path / "emb"), 0), 0, n_docs, "cpu").float().numpy()
    assert rows.shape == (n_docs, 768)
    # the query reps exactly as evaluate made them (one tower pass per query window)
    with torch.no_grad():
        qr = torch.cat([tr._encode_window(w) for w in tr._query_windows(ql)]).float().cpu()
    q = qr.to(torch.bfloat16).float().numpy()
    es, ei = orc.ip_topk(q, rows, k)   # fp64: the canonical order (ties by ascending id)
    assert tr.index.local.order_uncertified == 0
    if files:
        got = {}
        with open(tmp_path / "ret" / "0.0.json", encoding="utf-8") as f:
            for line in f:
                r = json.loads(line)
                got.setdefault(r["query_id"], []).append(r["doc_id"])
        for qi in range(n_q):
            # north_star: bit-exact retrieved doc ids and ranks against the fp64 evaluator
            assert len(got[qi]) == k
            np.testing.assert_array_equal(np.asarray(got[qi]), ei[qi])
    with open(tmp_path / "idx" / "0.docid.txt", encoding="utf-8") as f:
        assert json.load(f)["id"] == list(range(n_docs))
    pos = np.zeros((n_q, k), np.int8)
    for qi in range(n_q):
        for j in range(k):
            pos[qi, j] = has_answers(corpus[ei[qi, j]]["original"], answers[qi])
    # get_metrics per LOADER batch (its NDCG is a batch-level ratio), summed, / query_num
    ref = {}
    for a0 in range(0, n_q, bs):
        for key, v in get_metrics(pos[a0: a0 + bs], topk).items():
            ref[key] = ref.get(key, 0.0) + v
    for key, v in ref.items():
        assert abs(m[key] - v / n_q) < 1e-9, (key, m[key], v / n_q)
    with open(tmp_path / "cache" / "0.0_metrics", encoding="utf-8") as f:
        assert json.load(f)["query_num"] == n_q
