"""Answer matching used by Trainer.evaluate — restates DRT/evaluator/nq_eval.py:145-218
(SimpleTokenizer + has_answers: NFD-normalise, tokenise with the
[\\p{L}\\p{N}\\p{M}]+ | [^\\p{Z}\\p{C}] pattern, uncased contiguous token match).
CPU string work, outside the GPU hot path."""
from __future__ import annotations

import re
import unicodedata

import numpy as np
import regex

from .. import _native

_TOKEN_RE = regex.compile(r"([\p{L}\p{N}\p{M}]+)|([^\p{Z}\p{C}])",
                          flags=regex.IGNORECASE + regex.UNICODE + regex.MULTILINE)


def tokenize_uncased(text: str):
    return [m.group().lower() for m in _TOKEN_RE.finditer(text)]


# the same pattern without capture groups: findall returns the token strings directly
_TOKEN_FINDALL = regex.compile(r"[\p{L}\p{N}\p{M}]+|[^\p{Z}\p{C}]",
                               flags=regex.IGNORECASE + regex.UNICODE + regex.MULTILINE)
# passage separator of the bulk tokeniser: a punctuation character (one token of its own under
# the pattern, never part of a word token); a batch whose texts contain it is tokenised per text
_SEP = "\u2042"


def tokenize_uncased_many(texts):
    """[tokenize_uncased(NFD(t)) for t in texts] in one regex pass over the joined texts."""
    if not texts:
        return []
    if any(_SEP in t for t in texts):
        return [tokenize_uncased(unicodedata.normalize("NFD", t)) for t in texts]
    toks = _TOKEN_FINDALL.findall(unicodedata.normalize("NFD", _SEP.join(texts)))
    out, cur = [], []
    for t in toks:
        if t == _SEP:
            out.append(cur)
            cur = []
        else:
            cur.append(t.lower())
    out.append(cur)
    return out


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


class RowAnswerMatcher:
    """``has_answers`` for a whole query batch's retrieved ROWS at once (Trainer.evaluate).

    Same result as ``has_answers(text_of(row), answers[i])`` for every (query i, rank j) with
    ``row = rows[i, j] >= 0`` (pads get 0).  A row is tokenised at most once per evaluation (NFD,
    the uncased SimpleTokenizer pattern, one regex pass over many passages) into int32 token ids
    stored in a compact SLOT of a padded [slots, width] matrix (-1 pads, width grows with the
    longest passage seen); ``slot[row]`` maps an index row to its slot (-1 = not tokenised yet).
    Memory therefore follows the rows actually tokenised -- the corpus rows prefilled during the
    encode (up to the caller's budget) plus the rows queries retrieve -- not the corpus size.  A
    query's k passages are ONE slot gather, and an answer of n tokens is found by n shifted
    vectorised comparisons (a match never spans two passages; an empty answer matches every
    passage, as the reference's loop does).  ``version`` changes whenever ``tok`` is reallocated
    (the device mirror re-uploads on a change)."""

    def __init__(self, n_rows: int):
        self.vocab = {}
        self.n_rows = int(n_rows)
        self.width = 16
        self.slot = np.full(self.n_rows, -1, dtype=np.int64)
        self.tok = np.full((0, self.width), -1, dtype=np.int32)
        self.n_slots = 0
        self.version = 0
        self.n_filled = 0        # rows of [0, n_valid) that have a slot (fill's fast exit when all do)
        self.n_valid = self.n_rows   # rows the index really has (n_rows grows geometrically past it)
        self.slot_version = 0    # bumped whenever ``slot`` changes
        self.slot_epoch = 0      # bumped when ``slot`` is reallocated or rebased (a mirror re-uploads it whole)
        self.slot_log = []       # (rows, slots) assigned by each fill since: a mirror applies only these

    @property
    def seen(self) -> np.ndarray:
        return self.slot >= 0

    @property
    def token_bytes(self) -> int:
        return int(self.n_slots) * self.width * 4

    def ensure_rows(self, n_rows: int):
        """Rows [0, n_rows) addressable (geometric growth: called once per corpus batch)."""
        self.n_valid = max(self.n_valid, int(n_rows))
        if n_rows > self.n_rows:
            n_rows = max(int(n_rows), self.n_rows + self.n_rows // 2)
            sl = np.full(n_rows, -1, dtype=np.int64)
            sl[: self.n_rows] = self.slot
            self.slot, self.n_rows = sl, int(n_rows)
            self.slot_version += 1
            self.slot_epoch += 1
            self.slot_log = []

    def rebase(self, offset: int, n_local: int, n_total: int):
        """Move rows [0, n_local) (a shard tokenised by local row) to [offset, offset + n_local) of
        an n_total-row matcher (global rows of the sharded index).  The token slots stay put."""
        sl = np.full(n_total, -1, dtype=np.int64)
        sl[offset: offset + n_local] = self.slot[:n_local]
        self.slot, self.n_rows = sl, int(n_total)
        self.n_valid = int(n_total)
        self.n_filled = int((sl >= 0).sum())
        self.slot_version += 1
        self.slot_epoch += 1
        self.slot_log = []

    def _reserve(self, n_slots: int, width: int):
        cap, w = self.tok.shape[0], self.width
        while w < width:
            w *= 2
        if n_slots <= cap and w == self.width:
            return
        cap = max(n_slots, cap + cap // 2, 1024)
        t = np.full((cap, w), -1, dtype=np.int32)
        t[: self.n_slots, : self.width] = self.tok[: self.n_slots]
        self.tok, self.width = t, w
        self.version += 1

    def fill(self, rows, text_of) -> int:
        """Tokenise every row of ``rows`` not tokenised yet (``text_of(row)`` -> passage text)."""
        if self.n_filled >= self.n_valid:   # every row tokenised (the corpus prefill): nothing to look up
            return 0
        r = np.asarray(rows).reshape(-1)
        r = r[r >= 0]
        miss = r[self.slot[r] < 0]          # a gather; np.unique only over the (usually no) misses
        if miss.size:
            miss = np.unique(miss)
            v = self.vocab
            toks_list = tokenize_uncased_many([text_of(r) for r in miss.tolist()])
            mx = max((len(t) for t in toks_list), default=0)
            s0 = self.n_slots
            self._reserve(s0 + miss.size, mx)
            for j, toks in enumerate(toks_list):
                if toks:
                    self.tok[s0 + j, : len(toks)] = [v[t] if t in v else v.setdefault(t, len(v)) for t in toks]
            self.slot[miss] = np.arange(s0, s0 + miss.size)
            self.n_slots = s0 + int(miss.size)
            self.n_filled += int(miss.size)
            self.slot_version += 1
            self.slot_log.append((miss, s0))
        return int(miss.size)

    def _answer_ids(self, answers_i):
        """(token-id lists of the answers that can match, every): unknown tokens or answers longer
        than the width never match; an empty answer matches every passage."""
        out = []
        cache = self.__dict__.setdefault("_ans_words", {})
        if len(cache) > 1 << 20:
            cache.clear()
        for ans in answers_i:
            aw = cache.get(ans)
            if aw is None:   # tokenised once per distinct answer string (the vocabulary lookup is not
                aw = cache[ans] = tokenize_uncased(unicodedata.normalize("NFD", ans))   # cached: it grows)
            if not aw:
                return [], True
            ids = [self.vocab.get(w, -2) for w in aw]
            if min(ids) < 0 or len(ids) > self.width:
                continue
            out.append(ids)
        return out, False

    def match_rows(self, rows: np.ndarray, text_of, answers) -> np.ndarray:
        """int8 [B, k]: 1 where the passage at rows[i, j] contains any of answers[i]."""
        B, k = rows.shape
        hit = np.zeros((B, k), dtype=np.int8)
        if B == 0 or k == 0:
            return hit
        self.fill(rows, text_of)
        valid = rows >= 0
        W = self.width
        for i in range(B):
            lists, every = self._answer_ids(answers[i])
            if every:
                hit[i] = 1
                continue
            toks = None
            for ids in lists:
                n = len(ids)
                if toks is None:
                    toks = self.tok[self.slot[np.where(valid[i], rows[i], 0)]] if valid[i].any() \
                        else np.full((k, W), -1, np.int32)                        # [k, W] slot gather
                m = toks[:, : W - n + 1] == ids[0]
                for j in range(1, n):
                    m &= toks[:, j: W - n + 1 + j] == ids[j]
                hit[i] |= m.any(axis=1).astype(np.int8)
        hit[~valid] = 0
        return hit


# limits of drt_hit_metrics_i8 (csrc/match.hip kMetricMaxK / kMetricMaxB / kMetricMaxT)
METRICS_MAX_K = 2048
METRICS_MAX_B = 4096
METRICS_MAX_T = 16


class DeviceRowMatcher:
    """RowAnswerMatcher with the token slots resident in HBM: a query batch's k retrieved rows are
    gathered and compared on the GPU (the host only tokenises the batch's answers and any row not
    tokenised yet), on a stream of its own so the matching of batch j runs beside the search of
    batch j + 1.  Same result as ``RowAnswerMatcher.match_rows`` (the host matcher owns the
    vocabulary, the slots and the passage tokenisation); tests/test_answers_gpu.py compares the two.

    Per batch ONE kernel (drt_answer_match_i32, csrc/match.hip): wave (i, j) takes the token slot of
    retrieved row j of query i, its lanes take window starts s, and the row matches when some answer
    a of query i has toks[s + t] == ids[a][t] for every t < len(a) (s + len(a) <= W).  The host
    builds the batch's [B, A, n_max] answer ids (cached per answer string) and the slot array.
    (Round 3 evaluated [B, a, k, W] window masks with ~5 torch ops per answer token; the host cost of
    issuing them bounded the C2 query stage.)"""

    def __init__(self, host: "RowAnswerMatcher", device):
        import torch
        self.h = host
        self.device = torch.device(device)
        self.tok = None
        self._version = None
        self._slots = 0
        self.slot_dev = None
        self._slot_epoch = None
        self._log_i = 0
        # high priority: a stream of its own hardware-queue class, so a batch's comparison kernels never
        # queue behind the query tower pass the host enqueued on the compute stream meanwhile
        self.stream = torch.cuda.Stream(self.device, priority=-1)

    def _upload(self):
        """Mirror the host token matrix and row -> slot table: whole after a reallocation (version /
        epoch change), else only what the fills since the last upload added (new token slots; the
        newly assigned rows' slots scattered into the device table, not an O(rows) re-upload)."""
        import torch
        h = self.h
        with torch.cuda.stream(self.stream):
            if h.version != self._version or self.tok is None:
                self.tok = torch.from_numpy(np.ascontiguousarray(h.tok)).to(self.device)
                self._version = h.version
            elif h.n_slots > self._slots:
                a, b = self._slots, h.n_slots
                self.tok[a:b] = torch.from_numpy(np.ascontiguousarray(h.tok[a:b])).to(self.device)
            if h.slot_epoch != self._slot_epoch or self.slot_dev is None:
                self.slot_dev = torch.from_numpy(np.ascontiguousarray(h.slot)).to(self.device)
                self._slot_epoch = h.slot_epoch
                self._log_i = len(h.slot_log)
            elif self._log_i < len(h.slot_log):
                new = h.slot_log[self._log_i:]
                rows = np.concatenate([r for r, _ in new])
                slots = np.concatenate([np.arange(s0, s0 + r.size, dtype=np.int64) for r, s0 in new])
                rd = torch.from_numpy(rows.astype(np.int64)).pin_memory().to(self.device, non_blocking=True)
                sd = torch.from_numpy(slots).pin_memory().to(self.device, non_blocking=True)
                self.slot_dev.index_copy_(0, rd, sd)
                self._log_i = len(h.slot_log)
        self._slots = h.n_slots

    def match_rows(self, rows: np.ndarray, text_of, answers) -> np.ndarray:
        return self.match_rows_async(rows, text_of, answers).get()

    def match_rows_async(self, rows: np.ndarray, text_of, answers) -> "_PendingMatch":
        """match_rows enqueued on the matcher's stream; ``.get()`` waits for it (Trainer.evaluate
        reads batch j's matches after enqueueing batch j + 1's, so the host never waits for the
        comparison kernels of the batch it just handed over)."""
        import torch
        B, k = rows.shape
        if B == 0 or k == 0:
            return _PendingMatch(np.zeros((B, k), dtype=np.int8), None)
        hit = self._enqueue_hits(rows, text_of, answers)
        if hit is None:   # no row tokenised: every retrieved row is a pad
            return _PendingMatch(np.zeros((B, k), dtype=np.int8), None)
        with torch.cuda.stream(self.stream):
            out = torch.empty((B, k), dtype=torch.int8, pin_memory=True)
            out.copy_(hit, non_blocking=True)
            done = torch.cuda.Event()
            done.record(self.stream)
        return _PendingMatch(out, done)

    def match_metrics(self, rows, text_of, answers, topk_dev, acc) -> None:
        """The batch's answer matches AND its get_metrics (DRT/evaluator/metrics.py:4-59) added to the
        device sums ``acc`` [3 T] fp64 (recall, mrr, ndcg per cut-off of ``topk_dev`` [T] int32) on the
        matcher's stream -- nothing is read back per batch (drt_hit_metrics_i8).  ``rows``: the
        retrieved index rows [B, k], host int64 or a device tensor (Trainer.evaluate hands over the
        search's device ids; the host copy is taken only if some row still needs tokenising)."""
        import torch
        B, k = rows.shape
        if B == 0:
            return
        hit = self._enqueue_hits(rows, text_of, answers)
        T = int(topk_dev.numel())
        if k > METRICS_MAX_K or B > METRICS_MAX_B or T > METRICS_MAX_T:
            # beyond the kernel's LDS-resident limits (k up to 32768 on the large-k search path, huge
            # loader batches, many cut-offs): this batch's get_metrics on the host, added to the same sums
            from .metrics import get_metrics
            pos = np.zeros((B, k), dtype=np.int8) if hit is None else self._host_hits(hit)
            topk = [int(x) for x in topk_dev.cpu().tolist()]
            m = get_metrics(pos, topk)
            vals = [m[f"Recall@{t}"] for t in topk] + [m[f"MRR@{t}"] for t in topk] + [m[f"NDCG@{t}"] for t in topk]
            with torch.cuda.stream(self.stream):
                acc.add_(torch.tensor(vals, dtype=torch.float64).to(self.device, non_blocking=False))
            return
        with torch.cuda.stream(self.stream):
            if hit is None:
                hit = torch.zeros((B, k), dtype=torch.int8, device=self.device)
            _native.check(_native.load().drt_hit_metrics_i8(hit.data_ptr(), B, k, topk_dev.data_ptr(),
                                                             int(topk_dev.numel()), acc.data_ptr(),
                                                             self.stream.cuda_stream), "drt_hit_metrics_i8")

    def _host_hits(self, hit):
        """The device hit matrix [B, k] read back (the matcher's stream drained)."""
        import torch
        with torch.cuda.stream(self.stream):
            out = hit.cpu()
        return out.numpy()

    def _enqueue_hits(self, rows, text_of, answers):
        """hit [B, k] int8 on the device (the matcher's stream), or None when no row has tokens."""
        import torch
        B, k = rows.shape
        h = self.h
        on_dev = isinstance(rows, torch.Tensor)
        if h.n_filled < h.n_valid:   # rows without tokens yet: the host tokenises them first
            h.fill(rows.cpu().numpy() if on_dev else rows, text_of)
        self._upload()
        W = h.width
        lists, every = [], np.zeros(B, dtype=bool)
        for i in range(B):
            ids_i, every[i] = h._answer_ids(answers[i])
            lists.append(ids_i)
        A = max(1, max(len(x) for x in lists))
        n_max = max([1] + [len(a) for x in lists for a in x])
        ans = np.full((B, A, n_max), -3, dtype=np.int32)
        alen = np.zeros((B, A), dtype=np.int32)
        for i, x in enumerate(lists):
            for a, ids in enumerate(x):
                ans[i, a, : len(ids)] = ids
                alen[i, a] = len(ids)
        if h.n_slots == 0:
            return None
        lib = _native.load()
        dev = self.device
        if on_dev:   # the search's ids: produced on the index's stream, read on the matcher's
            self.stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(self.stream):
            if on_dev:
                r = rows.contiguous()
                r.record_stream(self.stream)
            else:   # the retrieved rows go up as they are; the kernel maps row -> token slot on the device
                r = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.int64)).pin_memory().to(dev, non_blocking=True)
            # answers and flags in one pinned upload
            meta = np.concatenate([ans.reshape(-1), alen.reshape(-1), every.astype(np.int32)])
            mt = torch.from_numpy(meta).pin_memory().to(dev, non_blocking=True)
            at, lt = mt[: ans.size], mt[ans.size: ans.size + alen.size]
            ev = mt[ans.size + alen.size:].to(torch.uint8)
            hit = torch.empty((B, k), dtype=torch.int8, device=dev)
            # one launch: wave (i, j) scans retrieved row j of query i for every answer of query i
            _native.check(lib.drt_answer_match_i32(self.tok.data_ptr(), W, r.data_ptr(), self.slot_dev.data_ptr(),
                                                   int(self.slot_dev.numel()), B, k, at.data_ptr(), lt.data_ptr(),
                                                   A, n_max, ev.data_ptr(), hit.data_ptr(),
                                                   self.stream.cuda_stream), "drt_answer_match_i32")
        return hit


class _PendingMatch:
    """pos_index of one batch behind an event (DeviceRowMatcher.match_rows_async)."""
    __slots__ = ("out", "done")

    def __init__(self, out, done):
        self.out, self.done = out, done

    def get(self) -> np.ndarray:
        if self.done is None:
            return self.out
        self.done.synchronize()
        return self.out.numpy().copy()
