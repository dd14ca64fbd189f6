"""GPU: DeviceRowMatcher (Trainer.evaluate's answer matching with the token matrix in HBM) equals
the host RowAnswerMatcher -- itself pinned to the reference's has_answers (tests/test_answers_cpu.py)
-- on random cases (pads, unknown tokens, empty answers, multi-token answers, growing widths)
and on the reference-generated golden cases."""
import json
import os

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("max_words", [40, 300])
def test_device_matcher_equals_host_random(dev, max_words):
    """max_words 300: token rows wider than a wave (several window starts per lane)."""
    from denseretrievaltoolkits_amd.evaluator.nq_eval import DeviceRowMatcher, RowAnswerMatcher, has_answers
    rng = np.random.default_rng(7)
    vocab = ["a", "b", "c", "d", "A", "b.", "c-d", "e", "É", "naïve", "⁂", "日本"]
    docs = [" ".join(rng.choice(vocab, size=int(rng.integers(0, max_words)))) for _ in range(500)]
    host = RowAnswerMatcher(0)
    host.ensure_rows(500)
    dm = DeviceRowMatcher(host, dev)
    ref_m = RowAnswerMatcher(0)
    ref_m.ensure_rows(500)
    for it in range(40):
        if it == 20:   # the row table grows mid-way: the mirror re-uploads it once, then scatters again
            host.ensure_rows(900)
            ref_m.ensure_rows(900)
        B, k = int(rng.integers(1, 9)), int(rng.integers(1, 60))
        rows = rng.integers(-1, 500, size=(B, k))
        ans = [[" ".join(rng.choice(vocab + ["zzz"], size=int(rng.integers(0, 5))))
                for _ in range(int(rng.integers(1, 4)))] for _ in range(B)]
        got = dm.match_rows(rows, lambda r: docs[r], ans)
        want = ref_m.match_rows(rows, lambda r: docs[r], ans)
        assert got.dtype == np.int8 and np.array_equal(got, want), it
        if it % 10 == 0:
            ref = [[int(has_answers(docs[r], ans[i])) if r >= 0 else 0 for r in rows[i]] for i in range(B)]
            assert got.tolist() == ref
    # the device row -> slot table was kept in step by scatters of each fill's new rows
    assert np.array_equal(dm.slot_dev.cpu().numpy(), host.slot)


def test_device_matcher_reference_golden(dev):
    from denseretrievaltoolkits_amd.evaluator.nq_eval import DeviceRowMatcher, RowAnswerMatcher
    with open(os.path.join(REPO, "tests", "golden", "answers.json"), encoding="utf-8") as f:
        g = json.load(f)
    dm = DeviceRowMatcher(RowAnswerMatcher(len(g["docs"])), dev)
    for c in g["cases"]:
        rows = np.array([c["docs"] + [-1, -1]], dtype=np.int64)
        got = dm.match_rows(rows, lambda r: g["docs"][r], [c["answers"]])
        assert got[0].tolist() == c["has"] + [0, 0], c


@pytest.mark.parametrize("B,k,topk", [(128, 1000, [1, 5, 20, 100, 1000]), (7, 50, [1, 3, 100]), (1, 1, [1, 2]),
                                      (300, 64, [64, 10])])
def test_device_metrics_equal_get_metrics(dev, B, k, topk):
    """drt_hit_metrics_i8 adds each batch's get_metrics (DRT/evaluator/metrics.py:4-59 restated in
    evaluator/metrics.py, pinned by tests/golden/metrics.json) to device sums: rows without hits, cut-offs
    beyond k, several batches accumulated."""
    import torch
    from denseretrievaltoolkits_amd import _native
    from denseretrievaltoolkits_amd.evaluator.metrics import get_metrics
    rng = np.random.default_rng(B + k)
    acc = torch.zeros(3 * len(topk), dtype=torch.float64, device=dev)
    tk = torch.tensor(topk, dtype=torch.int32, device=dev)
    ref = {}
    for it in range(3):
        hit = (rng.random((B, k)) < [0.0, 0.002, 0.05][it]).astype(np.int8)
        hit[0] = 0
        ht = torch.from_numpy(hit).to(dev)
        _native.check(_native.load().drt_hit_metrics_i8(ht.data_ptr(), B, k, tk.data_ptr(), len(topk), acc.data_ptr(),
                                                        _native.stream_ptr(dev)), "drt_hit_metrics_i8")
        for key, v in get_metrics(hit, topk).items():
            ref[key] = ref.get(key, 0.0) + v
    got = acc.cpu().numpy()
    T = len(topk)
    for t, kk in enumerate(topk):
        assert got[t] == ref[f"Recall@{kk}"]
        assert abs(got[T + t] - ref[f"MRR@{kk}"]) <= 1e-12 * max(1.0, abs(ref[f"MRR@{kk}"]))
        assert abs(got[2 * T + t] - ref[f"NDCG@{kk}"]) <= 1e-12 * max(1.0, abs(ref[f"NDCG@{kk}"]))
