"""CPU: pin the oracle and the host-side mirrors against the reference's golden vectors."""
import json
import os

import numpy as np
import pytest

from conftest import REPO
from oracle import bert_weights as bw
from oracle import search_oracle as orc

G = os.path.join(REPO, "tests", "golden")


def test_metrics_match_reference():
    from denseretrievaltoolkits_amd.evaluator.metrics import get_metrics
    for case in json.load(open(os.path.join(G, "metrics.json"))):
        hits = np.array(case["hits"], dtype=np.int8)
        got = get_metrics(hits, case["topk"])
        for k, v in case["metrics"].items():
            if isinstance(v, float) and np.isnan(v):
                assert np.isnan(got[k])
            else:
                assert got[k] == pytest.approx(v, rel=1e-12, abs=1e-12), k


def _merge_case_arrays(case):
    parts = case["results"]
    qids = sorted(parts[0].keys())
    per = max(len(p[q]) for p in parts for q in qids)
    nparts, nq = len(parts), len(qids)
    s = np.full((nparts, nq, per), orc.PAD_SCORE, np.float32)
    i = np.full((nparts, nq, per), -1, np.int64)
    for a, p in enumerate(parts):
        for r, q in enumerate(qids):
            items = sorted(((float(v), int(d[1:])) for d, v in p[q].items()), key=lambda x: (-x[0], x[1]))
            s[a, r, :len(items)] = [x[0] for x in items]
            i[a, r, :len(items)] = [x[1] for x in items]
    return qids, s, i


def test_partition_merge_matches_reference_merge():
    """oracle.merge_topk == merge_retrieval_results_by_score (utils.py:215-229) on distinct scores."""
    for case in json.load(open(os.path.join(G, "merge.json"))):
        qids, s, i = _merge_case_arrays(case)
        ms, mi = orc.merge_topk(s, i, case["topk"])
        for r, q in enumerate(qids):
            want = [int(d[1:]) for d, _ in case["merged"][q]]
            assert list(mi[r, :len(want)]) == want


def test_oracle_scores_are_reference_score_matrix():
    """The oracle's top-k scores are entries of DRModel.forward's q.p^T (biencoder.py:107)."""
    z = np.load(os.path.join(G, "loss.npz"))
    for name in ("n2", "n8"):
        q, p, sc = z[f"{name}_q"], z[f"{name}_p"], z[f"{name}_scores"]
        s, i = orc.ip_topk(q, p, p.shape[0])
        for r in range(q.shape[0]):
            np.testing.assert_allclose(s[r], sc[r][i[r]], rtol=1e-5, atol=1e-4)
            assert np.all(np.diff(s[r]) <= 0)


def test_oracle_corpus_topk_matches_reference_merge():
    """oracle.ip_topk over a 20k-row corpus at k = 1000 == the reference's own top-k
    (merge_retrieval_results_by_score over 3 row partitions, utils.py:215-229), ids and scores."""
    from helpers import corpus_topk_golden
    q, p, k, parts, ids, scores = corpus_topk_golden()
    s, i = orc.ip_topk(q, p, k)
    np.testing.assert_array_equal(i, ids)
    np.testing.assert_array_equal(s, scores)
    # and the oracle's partition merge of per-partition top-k lists
    bounds = np.linspace(0, p.shape[0], parts + 1).astype(int)
    ss, ii = [], []
    for a, b in zip(bounds[:-1], bounds[1:]):
        ps, pi = orc.ip_topk(q, p[a:b], k)
        ss.append(ps)
        ii.append(pi + a)
    ms, mi = orc.merge_topk(np.stack(ss), np.stack(ii), k)
    np.testing.assert_array_equal(mi, ids)


def _hf(layers, seed):
    import torch
    from transformers import BertModel
    torch.manual_seed(0)
    m = BertModel(bw.bert_config(layers=layers), add_pooling_layer=False).eval()
    return bw.init_model_(m, seed)


@pytest.mark.parametrize("tag", ["l2"])
def test_drmodel_mirror_torch_path_matches_reference_golden(tag):
    """The DRModel mirror's host semantics (pooling / head / normalize) equal the reference's (CPU, fp32)."""
    import torch
    from denseretrievaltoolkits_amd.model.biencoder import DRModelForInference
    from denseretrievaltoolkits_amd.model.linear import LinearHead
    z = np.load(os.path.join(G, f"encode_{tag}.npz"))
    lm = _hf(int(z["layers"]), int(z["seed"]))
    ids, mask = torch.from_numpy(z["input_ids"]), torch.from_numpy(z["attention_mask"])
    for key in [k for k in z.files if k.startswith("reps_")]:
        _, pooling, norm, head = key.split("_")
        h = None
        if head == "1":
            h = LinearHead(768, 768)
            with torch.no_grad():
                h.linear.weight.copy_(torch.from_numpy(bw.param_value(int(z["seed"]), "head.linear.weight", (768, 768))))
        m = DRModelForInference(lm_q=lm, lm_p=lm, pooling=pooling, head_q=h, head_p=h, normalize=norm == "1").eval()
        out = m(passage={"input_ids": ids, "attention_mask": mask})
        np.testing.assert_allclose(out.p_reps.numpy(), z[key], rtol=1e-4, atol=1e-5)


def test_rrmodel_mirror_torch_path_matches_reference_golden():
    import torch
    from denseretrievaltoolkits_amd.model.linear import LinearHead
    from denseretrievaltoolkits_amd.model.reranker import RRModel
    z = np.load(os.path.join(G, "rerank.npz"))
    lm = _hf(2, 2)
    head = LinearHead(768, 1)
    with torch.no_grad():
        head.linear.weight.copy_(torch.from_numpy(bw.param_value(2, "rr_head.linear.weight", (1, 768))))
    for pooling in ("first", "mean"):
        m = RRModel(lm=lm, head=head, pooling=pooling).eval()
        s = m(pos_pairs={"input_ids": torch.from_numpy(z["input_ids"]),
                         "attention_mask": torch.from_numpy(z["attention_mask"])})
        np.testing.assert_allclose(s.detach().numpy(), z[f"scores_{pooling}"], rtol=1e-4, atol=1e-5)
