"""Answer matching used by Trainer.evaluate — restates DRT/evaluator/nq_eval.py:145-218
(SimpleTokenizer + has_answers: NFD-normalise, tokenise with the
[\\p{L}\\p{N}\\p{M}]+ | [^\\p{Z}\\p{C}] pattern, uncased contiguous token match).
CPU string work, outside the GPU hot path."""
from __future__ import annotations

import re
import unicodedata

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
