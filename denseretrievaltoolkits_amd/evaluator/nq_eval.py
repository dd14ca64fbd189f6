"""Answer matching used by Trainer.evaluate — restates DRT/evaluator/nq_eval.py:145-218
(SimpleTokenizer + has_answers: NFD-normalise, tokenise with the
[\\p{L}\\p{N}\\p{M}]+ | [^\\p{Z}\\p{C}] pattern, uncased contiguous token match).
CPU string work, outside the GPU hot path."""
from __future__ import annotations

import re
import unicodedata

import numpy as np
import regex

_TOKEN_RE = regex.compile(r"([\p{L}\p{N}\p{M}]+)|([^\p{Z}\p{C}])",
                          flags=regex.IGNORECASE + regex.UNICODE + regex.MULTILINE)


def tokenize_uncased(text: str):
    return [m.group().lower() for m in _TOKEN_RE.finditer(text)]


def regex_match(text, pattern):
    try:
        pat = re.compile(pattern, flags=re.IGNORECASE + re.UNICODE + re.MULTILINE)
    except BaseException:
        return False
    return pat.search(text) is not None


def has_answers(text, answers, tokenizer=None, regex=False):
    text = unicodedata.normalize("NFD", text)
    if regex:
        return any(regex_match(text, unicodedata.normalize("NFD", a)) for a in answers)
    words = tokenize_uncased(text)
    for ans in answers:
        aw = tokenize_uncased(unicodedata.normalize("NFD", ans))
        n = len(aw)
        for i in range(0, len(words) - n + 1):
            if words[i:i + n] == aw:
                return True
    return False


class AnswerMatcher:
    """Vectorised ``has_answers`` over a query's whole retrieved list.

    The reference re-tokenises every retrieved passage for every query that
    retrieves it (Trainer.evaluate, DRT/trainer/trainer.py:302-321 -> nq_eval.py:203-218),
    Q·k regex tokenisations per evaluation.  Here each passage is tokenised once
    (cached by doc id) into int32 token ids; a query's k passages are laid end to
    end with a -1 separator, and each answer is found by narrowing the positions
    of its first token one token at a time (numpy), so a match can never span two
    passages.  Same result as ``has_answers(text, answers)`` for every (passage,
    query) pair: same NFD normalisation, same uncased tokeniser, contiguous token
    match, an empty answer matches every passage (as the reference's
    ``range(len(words) - 0 + 1)`` loop does).
    """

    def __init__(self):
        self.vocab = {}
        self._docs = {}

    def _ids(self, words):
        v = self.vocab
        out = np.empty(len(words), dtype=np.int32)
        for i, w in enumerate(words):
            t = v.get(w)
            if t is None:
                t = v[w] = len(v)
            out[i] = t
        return out

    def doc_tokens(self, doc_id, text) -> "np.ndarray":
        arr = self._docs.get(doc_id)
        if arr is None:
            arr = self._ids(tokenize_uncased(unicodedata.normalize("NFD", text)))
            self._docs[doc_id] = arr
        return arr

    def match(self, doc_ids, texts, answers) -> "np.ndarray":
        """int8 [len(doc_ids)]: 1 where passage j contains any answer."""
        m = len(doc_ids)
        hit = np.zeros(m, dtype=np.int8)
        if m == 0:
            return hit
        arrs = [self.doc_tokens(d, t) for d, t in zip(doc_ids, texts)]
        lens = np.fromiter((a.shape[0] + 1 for a in arrs), dtype=np.int64, count=m)
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
        flat = np.full(int(lens.sum()), -1, dtype=np.int32)
        for s, a in zip(starts, arrs):
            flat[s: s + a.shape[0]] = a
        for ans in answers:
            aw = tokenize_uncased(unicodedata.normalize("NFD", ans))
            if not aw:
                hit[:] = 1
                break
            ids = [self.vocab.get(w, -2) for w in aw]
            if min(ids) < 0:
                continue   # a token no passage has
            n = len(ids)
            pos = np.flatnonzero(flat[: flat.shape[0] - n + 1] == ids[0]) if flat.shape[0] >= n else np.empty(0, np.int64)
            for j in range(1, n):
                if pos.size == 0:
                    break
                pos = pos[flat[pos + j] == ids[j]]
            if pos.size:
                hit[np.searchsorted(starts, pos, side="right") - 1] = 1
        return hit
