"""Answer matching: the vectorised AnswerMatcher and the has_answers
restatement against golden vectors made by the REFERENCE's own
DRT/evaluator/nq_eval.py:203-218 has_answers (tools/gen_golden.py gen_answers)."""
import json
import os

import numpy as np

from denseretrievaltoolkits_amd.evaluator.nq_eval import AnswerMatcher, has_answers

GOLD = os.path.join(os.path.dirname(__file__), "golden", "answers.json")


def _gold():
    with open(GOLD, encoding="utf-8") as f:
        return json.load(f)


def test_has_answers_restatement_matches_reference_golden():
    g = _gold()
    for c in g["cases"]:
        got = [int(has_answers(g["docs"][j], c["answers"])) for j in c["docs"]]
        assert got == c["has"], c


def test_answer_matcher_matches_reference_golden():
    g = _gold()
    m = AnswerMatcher()
    for c in g["cases"]:
        texts = [g["docs"][j] for j in c["docs"]]
        got = m.match(c["docs"], texts, c["answers"])
        assert got.dtype == np.int8 and got.tolist() == c["has"], c


def test_answer_matcher_never_matches_across_passages():
    m = AnswerMatcher()
    # "rock" ends passage 0 and "roll" starts passage 1: only passage 2 holds "rock roll"
    got = m.match([0, 1, 2], ["we rock", "roll on", "rock roll"], ["Rock roll"])
    assert got.tolist() == [0, 0, 1]
    assert m.match([], [], ["x"]).tolist() == []
    assert m.match([5], [""], [""]).tolist() == [1]           # empty answer matches (reference loop)
    assert m.match([5], [""], ["a"]).tolist() == [0]


def test_answer_matcher_random_vs_has_answers():
    rng = np.random.default_rng(0)
    vocab = ["a", "b", "c", "d", "A", "b.", "c-d", "e"]
    m = AnswerMatcher()
    docs = [" ".join(rng.choice(vocab, size=int(rng.integers(0, 30)))) for _ in range(200)]
    for _ in range(300):
        ans = [" ".join(rng.choice(vocab, size=int(rng.integers(1, 4)))) for _ in range(int(rng.integers(1, 3)))]
        sel = rng.choice(200, size=50).tolist()
        got = m.match(sel, [docs[j] for j in sel], ans).tolist()
        assert got == [int(has_answers(docs[j], ans)) for j in sel]
