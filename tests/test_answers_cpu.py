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


def test_row_matcher_matches_reference_golden():
    """RowAnswerMatcher (Trainer.evaluate's batch matcher) on the reference-generated cases: each
    case is one query row of retrieved passages (pads appended: -1 rows match nothing)."""
    from denseretrievaltoolkits_amd.evaluator.nq_eval import RowAnswerMatcher
    g = _gold()
    m = RowAnswerMatcher(len(g["docs"]))
    for c in g["cases"]:
        rows = np.array([c["docs"] + [-1, -1]], dtype=np.int64)
        got = m.match_rows(rows, lambda r: g["docs"][r], [c["answers"]])
        assert got.dtype == np.int8 and got[0].tolist() == c["has"] + [0, 0], c


def test_row_matcher_random_vs_has_answers():
    from denseretrievaltoolkits_amd.evaluator.nq_eval import RowAnswerMatcher, tokenize_uncased, \
        tokenize_uncased_many
    import unicodedata
    rng = np.random.default_rng(1)
    vocab = ["a", "b", "c", "d", "A", "b.", "c-d", "e", "É", "naïve", "⁂", "日本"]
    docs = [" ".join(rng.choice(vocab, size=int(rng.integers(0, 40)))) for _ in range(300)]
    m = RowAnswerMatcher(0)
    m.ensure_rows(300)
    for _ in range(60):
        B, k = 4, 30
        rows = rng.integers(-1, 300, size=(B, k))
        ans = [[" ".join(rng.choice(vocab, size=int(rng.integers(0, 4)))) for _ in range(int(rng.integers(1, 3)))]
               for _ in range(B)]
        got = m.match_rows(rows, lambda r: docs[r], ans)
        ref = [[int(has_answers(docs[r], ans[i])) if r >= 0 else 0 for r in rows[i]] for i in range(B)]
        assert got.tolist() == ref
    # the bulk tokeniser equals the per-text one (also with the separator inside a text)
    assert tokenize_uncased_many(docs[:50]) == [tokenize_uncased(unicodedata.normalize("NFD", t)) for t in docs[:50]]
    # rebase: rows tokenised by local row land at the shard's global offset
    m2 = RowAnswerMatcher(0)
    m2.ensure_rows(10)
    m2.fill(np.arange(10), lambda r: docs[r])
    m2.rebase(100, 10, 200)
    rows = np.arange(100, 110)[None, :]
    got = m2.match_rows(rows, lambda r: (_ for _ in ()).throw(AssertionError("refilled")), [["a"]])
    assert got[0].tolist() == [int(has_answers(docs[r], ["a"])) for r in range(10)]


def test_row_matcher_memory_follows_tokenised_rows():
    """The token matrix holds only rows that were tokenised: a 5M-row index with 3 retrieved rows
    keeps a few KiB of tokens (the dense [rows, W] matrix did not scale to 21M)."""
    from denseretrievaltoolkits_amd.evaluator.nq_eval import RowAnswerMatcher
    m = RowAnswerMatcher(5_000_000)
    texts = {7: "the eiffel tower in paris", 4_999_999: "tokyo tower", 123: " ".join(["w"] * 40)}
    rows = np.array([[7, 4_999_999, 123, -1]])
    got = m.match_rows(rows, lambda r: texts[r], [["tower"]])
    assert got.tolist() == [[1, 1, 0, 0]]
    assert m.n_slots == 3 and m.width == 64 and m.tok.nbytes <= 1024 * 64 * 4
    v = m.version
    m.fill(np.array([8]), lambda r: " ".join(["x"] * 100))     # wider passage: reallocation
    assert m.version > v and m.width == 128 and m.match_rows(rows, None, [["tower"]]).tolist() == [[1, 1, 0, 0]]
