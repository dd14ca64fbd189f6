"""Device-resident exact inner-product indexes (faiss.IndexFlatIP replacement).

``FlatIPIndex``     one GPU: the corpus lives in HBM as bf16 rows; ``search``
                    runs the fused scan + top-k kernels (csrc/search.hip).
``ShardedFlatIP``   one process per GPU (torch.distributed, RCCL): rank r
                    owns a contiguous row shard; every rank scans its shard
                    for the same query batch, the per-shard top-k lists are
                    all-gathered over RCCL and merged on device
                    (SURVEY §8e).  Global id of a row = shard offset + local.

Reference behaviour replaced: faiss.IndexFlatIP (DRT/evaluator/index.py:19-33)
and the per-rank .npy files + rank-0 index file exchange of
Trainer._encoding_corpus/_index_corpus/_load_index (trainer.py:191-262).
Semantics kept: ``add`` appends rows with sequential ids, ``search(q, k)``
returns (D [nq,k] fp32, I [nq,k] int64) in descending score, missing rows as
(-FLT_MAX, -1).  Refinements: ties ordered by ascending id; storage is bf16.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from . import _native, comm, kernels, shards


def _as_device_bf16(x, device) -> torch.Tensor:
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(x))
    if not isinstance(x, torch.Tensor):
        raise TypeError(f"expected np.ndarray or torch.Tensor, got {type(x)}")
    return x.detach().to(device=device, dtype=torch.bfloat16).contiguous()


def _stage_host(*ts: torch.Tensor):
    """Host copies of device tensors, staged without waiting: pinned non-blocking D2H copies on
    the tensors' device stream plus one event behind them.  The host looks at them only when the
    work is finished, after the next batch has been enqueued, so reading them never drains the
    stream (the copies and the event go on the tensors' OWN device stream: an index may live on
    a device other than the current one)."""
    dev = ts[0].device
    hs = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in ts]
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev)
        for h, t in zip(hs, ts):
            h.copy_(t, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
    return hs, ev


def _stage_status(st: torch.Tensor):
    """Host copy of a device status vector (see _stage_host)."""
    if not st.is_cuda:
        return st, None
    (h,), ev = _stage_host(st)
    return h, ev


def _status_failed(h: torch.Tensor, ev) -> int:
    """Queries whose status bit 0 is set (not certified: redo exactly)."""
    if ev is not None:
        ev.synchronize()
    return int(((h & 1) != 0).sum().item())


def _order_uncertified(h: torch.Tensor) -> int:
    """Queries whose status bit 1 is set (canonical order not certified: fp32 order kept)."""
    return int(((h & 2) != 0).sum().item())


# Canonical order (kernels.refine): results ranked by the EXACT inner products (fp64 sums of the
# bf16 products, ties by ascending id) -- what an fp64 evaluator returns -- instead of by the
# scan's fp32 sums.  Costs one gather of the ~k candidate rows per query (~1.3 % of a 10M-row
# step).  False: the fp32 scan order (the bf16-product sums faiss-style, near-ties in MFMA order).
EXACT_ORDER = True


class _HostResult:
    """(scores, ids) of a batch copied to pinned host memory behind an event (to_host mode)."""
    __slots__ = ("hs", "ev")

    def __init__(self, s: torch.Tensor, i: torch.Tensor):
        self.hs, self.ev = _stage_host(s, i)

    def get(self, s: torch.Tensor, i: torch.Tensor, redone: bool):
        """numpy (scores, ids); a batch that was redone after staging is copied again."""
        if redone:
            return s.cpu().numpy(), i.cpu().numpy()
        self.ev.synchronize()
        return self.hs[0].numpy(), self.hs[1].numpy()


def _pipeline(batches, enqueue, finish):
    """Enqueue batch j + 1 before finishing (certifying) batch j; yields finished results in order."""
    pend = None
    for j, q in enumerate(batches):
        cur = enqueue(j, q)
        if pend is not None:
            yield finish(pend)
        pend = cur
    if pend is not None:
        yield finish(pend)


# Batched search (search_batches): the per-batch fixed costs of the global-threshold protocol --
# the sample scan + its k-th selection and, across shards, the sample-list all-gather, the packed
# all-gather and the merge -- are paid once per GROUP of query batches; every batch still streams
# the whole shard once in its own filter scan.  Queries per group (16 batches of 128):
GROUP_QUERIES = 2048
# one-GPU indexes take the grouped path from this many rows up (round 2/3 it was off: the group's
# blocks then ran one after another and the back-to-back filter scans measured 2-3 % slower,
# profiles/r02j_bench_*.json; across GPUs the group also saves two collectives per batch)
GROUP_MIN_ROWS = 500_000
# A group's filter launch runs its 16 query blocks side by side on each XCD (csrc/search.hip
# launch_scan_d) and a corpus tile is fetched from HBM once for all of them while they stay within the
# XCD's 4 MB L2 of each other.  Over a long shard they drift apart (10M rows: 2.13-2.33 ms per batch, no
# better than 16 per-batch launches), so a one-GPU index runs the group's filter as one launch per row
# chunk of at most this many rows, each chunk's packed lists a part of the merge like the shards of a
# sharded index (round 5: 10M rows 1.90 vs 2.13 ms per batch, tools/group_chunk_probe.py,
# profiles/r05g/; 1.25M rows is also the W = 8 shard).
GROUP_CHUNK_ROWS = 1_250_000


def group_chunks(nrows: int, chunk_rows: int = None, nch: int = None):
    """Row ranges [(a, b)] of a group filter: balanced chunks of <= chunk_rows rows, or exactly ``nch``
    chunks (a sharded index: every rank splits its shard into the same count, so the ranks' part buffers
    have one shape; a chunk may be empty)."""
    chunk_rows = GROUP_CHUNK_ROWS if chunk_rows is None else chunk_rows
    if nch is None:
        if chunk_rows <= 0 or nrows <= chunk_rows:
            return [(0, nrows)]
        nch = -(-nrows // chunk_rows)
    if nch <= 1:
        return [(0, nrows)]
    per = -(-nrows // nch)
    return [(min(nrows, c * per), min(nrows, (c + 1) * per)) for c in range(nch)]


def _groups(batches, cap=None):
    cap = GROUP_QUERIES if cap is None else cap
    grp, n = [], 0
    for q in batches:
        if grp and n + q.shape[0] > cap:
            yield grp
            grp, n = [], 0
        grp.append(q)
        n += q.shape[0]
    if grp:
        yield grp


def _reserve_group_memory(local, k: int, n_global: int, chunks=None):
    """Size torch's caching allocator for a FULL group once per (index, k): the group's sample / filter
    workspace (~0.85 GB at 2048 queries over a 10M-row shard) and its result lists are carved from one
    segment allocated here, so the first full group after shorter ones (a short warm-up, a small first
    batch set) does not hipMalloc inside the search.  (Round 6: the driver's 20-step bench met its first
    2048-query group after a 640-query warm-up.)"""
    key = (k, n_global, GROUP_QUERIES)
    if getattr(local, "_group_reserved", None) == key or local.ntotal == 0:
        return
    kc = kernels.refine_width(k)
    nq = GROUP_QUERIES
    ws = int(_native.load().drt_ip_topk_dist_workspace(nq, local.ntotal, n_global, local.dp, kc))
    nparts = max(1, len(chunks or [0]))
    lists = nq * (kc + 1) * 8 * (nparts + 1)                  # packed lists (+ the chunked form's parts)
    outs = nq * kc * (4 + 8 + 4) + nq * k * (4 + 8) * 2       # merge outputs, deltas, refined results
    need = ws + lists + outs + (64 << 20)
    with torch.cuda.device(local.device):
        blk = torch.empty(need, dtype=torch.uint8, device=local.device)
        del blk   # back to the cache as one free segment the group's allocations are split from
    local._group_reserved = key


class _SideChannel:
    """The exchange side channel of a sharded index (round 6, SURVEY §5 "overlap the exchange for batch i
    with the scan for batch i + 1"): a second HIP stream and a second communicator over the same ranks.
    A group's packed all-gather, merge and canonical-order stage (its delta all-reduce included) run on
    the side stream behind an event on the filter scan, while the next group's sample, sample-list
    all-gather and filter scans run on the compute stream.  The second communicator matters: one RCCL
    communicator runs its collectives in issue order on one internal stream, so the next group's
    sample-list all-gather would queue behind this group's exchange and hold its scans back."""
    __slots__ = ("stream", "group")

    def __init__(self, stream, group):
        self.stream, self.group = stream, group

    def gather(self, t: torch.Tensor) -> torch.Tensor:
        return comm.all_gather_stacked(t, self.group)

    def all_reduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        return comm.all_reduce_sum_(t, self.group)


def _gtau_enqueue_group(local, qs, k: int, n_global: int, offset: int, gather, to_host: bool = False,
                        stats=None, all_reduce_sum=None, id_shift: int = 0, chunks=None, world: int = 1,
                        side: _SideChannel = None):
    """One group of query batches through the global-threshold protocol (see ShardedFlatIP):
    ONE sample launch for all of the group's queries, one exchange of the sample lists, one
    threshold launch, one filter scan (+ select) per batch writing its packed top-k into a group buffer,
    one exchange of that buffer and one merge that certifies every query.  ``gather(t)`` ->
    [world, *t.shape] (identity stack on one GPU).  ``to_host``: the merged group's results are
    also staged to pinned host memory behind the merge.  ``stats`` (the GLOBAL row statistics):
    the shards keep kc = refine_width(k) candidates each, the merge keeps kc, and the canonical
    stage (kernels.refine, deltas summed across shards by ``all_reduce_sum``) orders the top-k.
    ``id_shift`` is added to every returned id (a one-GPU index searched with an id offset: the
    protocol itself runs on the index's own row numbers, packed in 32 bits).  ``chunks``: the filter runs as
    one launch per row range of this shard (group_chunks) and the chunks' hits are selected once
    (kernels.dist_filter_chunks_into; d > 768: each chunk's packed lists are a part of the merge, gathered
    [world, chunks, ...] -- the same chunk count on every rank).  ``side`` (a _SideChannel): everything
    after the filter scans -- exchange, merge, canonical stage, status staging -- goes on the side stream
    and through its communicator, so the caller can enqueue the next group's scans behind it."""
    sizes = [q.shape[0] for q in qs]
    qg = qs[0] if len(qs) == 1 else torch.cat(qs)
    best = local.dist_sample(qg, n_global, k)                       # [Qg, r]
    lists = gather(best).contiguous()                               # [world, Qg, r]
    tau = kernels.dist_tau(lists, k)                                # [Qg]: one launch for the group
    kc = kernels.refine_width(k) if stats is not None else k
    # entries each rank's list carries through the exchange (round 6: W > 1 ranks send their best
    # exchange_cap(kc, W) instead of kc; the merge certifies truncated lists, a failure is redone exactly)
    lc = kernels.exchange_cap(kc, world) if world > 1 and getattr(local, "exchange_capped", True) else kc
    if chunks is not None and len(chunks) > 1 and qg.shape[1] <= 768:
        # long shard: one filter launch per row chunk (the group's query blocks stay in step over a
        # chunk, so its tiles are read from HBM once), all chunks' hits in one list, one select
        lists = torch.empty((qg.shape[0], lc + 1), dtype=torch.int64, device=qg.device)
        starts = [a for a, _ in chunks] + [chunks[-1][1]]
        kernels.dist_filter_chunks_into(qg, local.rows, n_global, lc, offset, tau, starts, lists)
    elif chunks is not None and len(chunks) > 1:
        # (wider rows) one filter launch + select per chunk, every chunk's lists a part of the merge
        lists = torch.empty((len(chunks), qg.shape[0], kc + 1), dtype=torch.int64, device=qg.device)
        for c, (a, b) in enumerate(chunks):
            kernels.dist_filter_into(qg, local.rows[a:b], n_global, kc, offset + a, tau, lists[c])
    else:
        lists = torch.empty((qg.shape[0], lc + 1), dtype=torch.int64, device=qg.device)
        # ONE filter launch for the whole group (grid: corpus tiles x 128-query blocks, the blocks of
        # a tile co-located per XCD) and one select over all of its queries
        kernels.dist_filter_into(qg, local.rows, n_global, lc, offset, tau, lists)

    def exchange(gather, all_reduce_sum):
        allp = gather(lists)
        if lists.dim() == 3:
            allp = allp.reshape(-1, qg.shape[0], kc + 1)
        s, i, st = kernels.merge_packed(allp, kc, n_global, k_cert=k)
        if stats is not None:
            s, i = kernels.refine(qg, local.rows, offset, s, i, k, stats, tau, st, all_reduce_sum)
        if id_shift:
            i = torch.where(i >= 0, i + id_shift, i)
        h, ev = _stage_status(st)
        host = _HostResult(s, i) if to_host else None
        return s, i, st, h, ev, host

    if side is None:
        return (qs, sizes) + exchange(gather, all_reduce_sum)
    compute = torch.cuda.current_stream(qg.device)
    scanned = torch.cuda.Event()
    scanned.record(compute)
    with torch.cuda.stream(side.stream):
        side.stream.wait_event(scanned)
        for t in (lists, qg, tau):   # compute-stream allocations the side stream still reads
            t.record_stream(side.stream)
        s, i, st, h, ev, host = exchange(side.gather, side.all_reduce_sum)
    for t in (s, i, st):   # side-stream results the caller reads on its own stream
        t.record_stream(compute)
    return qs, sizes, s, i, st, h, ev, host


def _gtau_finish_group(pend, redo, wide=None):
    """Per-batch results of a group; a batch with an uncertified query is redone by ``redo(q)``
    (the exact path).  Every rank merged the same gathered lists, so all ranks redo the same
    batches (their collectives stay matched).  ``wide(q, s, i, st)`` (one GPU): the wide resolve of
    a batch's queries whose canonical order the candidate list could not certify (status 2), in
    place; returns how many it resolved.  With staged host copies the results are numpy.
    Returns (results, batches redone, queries left in the fp32 order)."""
    qs, sizes, s, i, st, h, ev, host = pend
    if ev is not None:
        ev.synchronize()
    bad = (h & 1) != 0
    wid = (h & 3) == 2
    res, o, nredo, nunc = [], 0, 0, 0
    hs = hi = None
    for q, nb in zip(qs, sizes):
        nw = int(wid[o:o + nb].sum()) if not bool(bad[o:o + nb].any()) else 0
        if nw and wide is not None:
            nunc += nw - wide(q, s[o:o + nb], i[o:o + nb], st[o:o + nb])
            res.append((s[o:o + nb].cpu().numpy(), i[o:o + nb].cpu().numpy()) if host is not None
                       else (s[o:o + nb], i[o:o + nb]))
        elif bool(bad[o:o + nb].any()):
            rs, ri = redo(q)
            res.append((rs.cpu().numpy(), ri.cpu().numpy()) if host is not None else (rs, ri))
            nredo += 1
        elif host is not None:
            nunc += nw
            if hs is None:
                hs, hi = host.get(s, i, False)
            res.append((hs[o:o + nb], hi[o:o + nb]))
        else:
            nunc += nw
            res.append((s[o:o + nb], i[o:o + nb]))
        o += nb
    return res, nredo, nunc


class _GroupPend:
    """One enqueued group of ``FlatIPIndex.enqueue_batches`` (its result, once finished)."""
    __slots__ = ("pend", "k", "id_offset", "res")

    def __init__(self, pend, k, id_offset):
        self.pend, self.k, self.id_offset, self.res = pend, k, id_offset, None


class _GroupMember:
    """Batch j of an enqueued group."""
    __slots__ = ("group", "j")

    def __init__(self, group, j):
        self.group, self.j = group, j


class FlatIPIndex:
    """Exact IP index over bf16 rows resident on one GPU (IndexFlatIP semantics).

    Any d <= 1024 (the scan keeps a query block's d values on chip; faiss's GPU flat index has the
    same kind of bound on k, none on d): rows and queries of a d that is not a multiple of 64 are
    stored zero-padded to the next multiple (``dp``), which leaves every inner product exactly
    unchanged.  ``rows`` is the padded [ntotal, dp] view the kernels scan."""

    def __init__(self, d: int, device=None, capacity: int = 0):
        if d <= 0 or d > 1024:
            raise ValueError(f"dimension {d} unsupported: the HIP scan needs 0 < d <= 1024")
        self.d = int(d)
        self.dp = (self.d + 63) // 64 * 64
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._buf = torch.zeros((max(0, capacity), self.dp), dtype=torch.bfloat16, device=self.device)
        self.ntotal = 0
        self.metric = "inner_product"
        self.exact_order = EXACT_ORDER
        self._stats = None     # row statistics of rows [0, _stats_n) (kernels.row_stats)
        self._stats_n = 0

    # faiss-compatible surface -----------------------------------------
    @property
    def is_trained(self) -> bool:
        return True

    def reset(self):
        self.ntotal = 0
        self._stats = None   # refilled rows must be rescanned (a stale max-norm / integer flag would
        self._stats_n = 0    # make the canonical stage's error bound wrong)

    def reserve(self, n: int):
        if n > self._buf.shape[0]:
            nb = torch.zeros((n, self.dp), dtype=torch.bfloat16, device=self.device)
            if self.ntotal:
                nb[: self.ntotal] = self._buf[: self.ntotal]
            self._buf = nb

    def add(self, x) -> None:
        x = _as_device_bf16(x, self.device)
        if x.dim() != 2 or x.shape[1] != self.d:
            raise ValueError(f"add: expected [n, {self.d}] rows, got {tuple(x.shape)}")
        n = x.shape[0]
        if self.ntotal + n > self._buf.shape[0]:
            self.reserve(max(self.ntotal + n, int(self._buf.shape[0] * 1.5) + 1))
        self._buf[self.ntotal: self.ntotal + n, : self.d] = x
        if self.dp != self.d:   # (the buffer may hold rows of an earlier, reset() index)
            self._buf[self.ntotal: self.ntotal + n, self.d:] = 0
        self.ntotal += n

    @property
    def rows(self) -> torch.Tensor:
        return self._buf[: self.ntotal]

    def row_stats(self) -> torch.Tensor:
        """Row statistics of the canonical-order stage (one pass over rows added since the last call)."""
        if self._stats is None or self._stats_n > self.ntotal:
            self._stats = kernels.row_stats(self.rows)
        elif self._stats_n < self.ntotal:
            self._stats = kernels.row_stats(self.rows[self._stats_n:], prev=self._stats)
        self._stats_n = self.ntotal
        return self._stats

    def _stats_arg(self):
        return self.row_stats() if self.exact_order and self.ntotal > 0 else None

    order_uncertified = 0   # queries whose canonical order could not be certified (fp32 order kept)

    @classmethod
    def from_rows(cls, rows: torch.Tensor) -> "FlatIPIndex":
        """Wrap an existing bf16 [n, d] device tensor as the index rows (no copy)."""
        if rows.dtype != torch.bfloat16 or rows.dim() != 2 or not rows.is_cuda:
            raise ValueError("from_rows expects a [n, d] bf16 device tensor")
        idx = cls(rows.shape[1], device=rows.device, capacity=0)
        idx._buf = idx._pad(rows).contiguous()
        idx.ntotal = rows.shape[0]
        return idx

    # search: the fast threshold path + certification.  A query the threshold path cannot
    # certify (status != 0, ~1e-9 per query on real data) is redone by the exact dense rescan.
    resolved = 0   # queries redone by the exact rescan over this index's lifetime

    def _enqueue(self, q, k: int, id_offset: int = 0, out=None, to_host: bool = False):
        qd = self._queries(q)
        stats = self._stats_arg()
        if stats is None and k > kernels.MAX_K:   # the large-k path always ranks exactly: reuse the index's stats
            stats = self.row_stats()
        s, i, st = kernels.ip_topk(qd, self.rows, k, id_offset=id_offset, resolve=False, out=out, stats=stats)
        h, ev = _stage_status(st)
        host = _HostResult(s, i) if to_host else None
        return qd, s, i, st, h, ev, id_offset, k, host, stats

    def _finish(self, pend):
        qd, s, i, st, h, ev, off, k, host, stats = pend
        nbad = _status_failed(h, ev)
        if nbad:
            self.resolved += kernels.resolve_failed(qd, self.rows, k, off, s, i, st, n_failed=nbad, stats=stats)
            h = st.cpu()   # the rescan set each redone query's status anew
        nwide = int(((h & 3) == 2).sum().item()) if stats is not None else 0
        nres = self._wide(qd, k, off, s, i, st, stats, nwide)
        self.order_uncertified += _order_uncertified(h) - nres
        if host is not None:
            return host.get(s, i, nbad > 0 or nres > 0)
        return s, i

    wide_resolved = 0   # queries put in the canonical order by the wide resolve (massive near-ties)
    range_resolved = 0  # ... of them, windows wider than 65,536 rows (kernels.exact_by_ranges)

    def _wide(self, qd, k, off, s, i, st, stats, nwide=None) -> int:
        """Wide resolve (kernels.resolve_wide) of the queries with status 2; returns how many it resolved."""
        if stats is None or nwide == 0:
            return 0
        n = kernels.resolve_wide(qd, self.rows, k, off, s, i, st, stats, n_wide=nwide)
        if n < (nwide if nwide is not None else n + 1):
            # windows wider than the wide resolve's 65,536 rows (round 6): exact top-k range by range
            left = torch.nonzero((st & 3) == 2).flatten()
            if left.numel():
                s2, i2 = kernels.exact_by_ranges(qd.index_select(0, left).contiguous(), self.rows, k, off, stats)
                s.index_copy_(0, left, s2)
                i.index_copy_(0, left, i2)
                st.index_fill_(0, left, 0)
                n += int(left.numel())
                self.range_resolved += int(left.numel())
        self.wide_resolved += n
        return n

    def search_exact_keys(self, q, k: int, id_offset: int = 0):
        """(exact order keys, ids) int64 [nq, k] of this index's canonical top-k (kernels.ip_topk_exact_keys):
        a shard's part of a sharded search at k > 2048, merged across shards by exact key."""
        return kernels.ip_topk_exact_keys(self._queries(q), self.rows, k, id_offset=id_offset, stats=self.row_stats())

    def search_unresolved(self, q, k: int, id_offset: int = 0):
        """(scores, ids, status) with status still on device (the per-shard protocol gathers it);
        the fp32 scan order (the per-shard lists are merged by their fp32 scores)."""
        return kernels.ip_topk(self._queries(q), self.rows, k, id_offset=id_offset, resolve=False)

    def search_device(self, q, k: int, id_offset: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
        return self._finish(self._enqueue(q, k, id_offset))

    group_fallbacks = 0   # batches of grouped searches redone by the exact per-batch path

    def search_batches(self, batches, k: int, id_offset: int = 0, outs=None):
        """Certified top-k of every query batch (device tensors), pipelined: the next batch (or
        group of batches) is enqueued before the host checks the previous one's status, so the
        certification costs an event wait on finished work, not a drained stream.  On a large
        shard the batches run in groups (GROUP_QUERIES): one sample launch and one merge per
        group, one filter scan per batch (_gtau_enqueue_group).  ``outs[j]`` = optional
        (scores, ids) output buffers of batch j (per-batch path).  This is the path
        BaseFaissIPRetriever.batch_search, Trainer.evaluate and bench.py time."""
        return list(self.search_batches_iter(batches, k, id_offset, outs))

    def _use_groups(self, k: int = 0) -> bool:
        # the grouped path packs row numbers into 32 bits (an id offset is added afterwards); k beyond
        # the candidate-list kernels' takes the per-batch large-k path (kernels.ip_topk)
        return k <= kernels.MAX_K and GROUP_MIN_ROWS <= self.ntotal < 0xFFFFFFFF

    def enqueue_batches(self, batches, k: int, id_offset: int = 0, to_host: bool = False) -> list:
        """Every batch's search enqueued now (in groups where ``search_batches`` would group them);
        collect each with ``finish_batch``."""
        if not self._use_groups(k):
            return [self._enqueue(q, k, id_offset, None, to_host) for q in batches]
        out = []
        stats = self._stats_arg()
        _reserve_group_memory(self, k, self.ntotal, group_chunks(self.ntotal))
        for g in _groups(list(batches)):
            gp = _GroupPend(_gtau_enqueue_group(self, [self._queries(q) for q in g], k, self.ntotal, 0,
                                                lambda t: t.unsqueeze(0), to_host, stats=stats, id_shift=id_offset,
                                                chunks=group_chunks(self.ntotal)),
                            k, id_offset)
            out += [_GroupMember(gp, j) for j in range(len(g))]
        return out

    def finish_batch(self, pend):
        """(scores, ids) of one ``enqueue_batches`` entry, certified (uncertified queries redone)."""
        if isinstance(pend, _GroupMember):
            gp = pend.group
            if gp.res is None:   # the group's certificates are checked once, by its first member
                stats = self._stats_arg()
                res, nredo, nunc = _gtau_finish_group(
                    gp.pend, lambda q: self.search_device(q, gp.k, gp.id_offset),
                    lambda q, s, i, st: self._wide(q, gp.k, gp.id_offset, s, i, st, stats))
                self.group_fallbacks += nredo
                self.order_uncertified += nunc
                gp.res = res
            return gp.res[pend.j]
        return self._finish(pend)

    def search_batches_iter(self, batches, k: int, id_offset: int = 0, outs=None, to_host: bool = False):
        """search_batches as a generator: batch j's result is yielded once batch j + 1 (or the next
        group) is on the GPU, so the caller's host work on batch j overlaps the device work on
        batch j + 1.  ``to_host``: yield numpy (scores, ids) from pinned copies staged behind each
        batch (no stream-draining .cpu() per batch)."""
        batches = list(batches)
        if outs is None and self._use_groups(k):
            yield from self._search_groups(batches, k, id_offset, to_host)
            return
        yield from _pipeline(batches, lambda j, q: self._enqueue(q, k, id_offset, outs[j] if outs else None,
                                                                 to_host), self._finish)

    def _search_groups(self, batches, k: int, id_offset: int, to_host: bool = False):
        groups = [[self._queries(q) for q in g] for g in _groups(batches)]

        def fin(pend):
            res, nredo, nunc = _gtau_finish_group(pend, lambda q: self.search_device(q, k, id_offset),
                                                  lambda q, s, i, st: self._wide(q, k, id_offset, s, i, st, stats))
            self.group_fallbacks += nredo
            self.order_uncertified += nunc
            return res

        stats = self._stats_arg()
        chunks = group_chunks(self.ntotal)
        _reserve_group_memory(self, k, self.ntotal, chunks)
        for res in _pipeline(groups, lambda j, g: _gtau_enqueue_group(self, g, k, self.ntotal, 0,
                                                                      lambda t: t.unsqueeze(0), to_host,
                                                                      stats=stats, id_shift=id_offset,
                                                                      chunks=chunks), fin):
            yield from res

    def search(self, q, k: int) -> Tuple[np.ndarray, np.ndarray]:
        s, i = self.search_device(q, k)
        return s.cpu().numpy(), i.cpu().numpy()

    # global-threshold protocol steps (ShardedFlatIP) ---------------------
    def _pad(self, x: torch.Tensor) -> torch.Tensor:
        return x if self.dp == self.d else torch.nn.functional.pad(x, (0, self.dp - self.d))

    def _queries(self, q):
        qd = _as_device_bf16(q, self.device)
        if qd.dim() != 2 or qd.shape[1] not in (self.d, self.dp):
            raise ValueError(f"search: expected [nq, {self.d}] queries, got {tuple(qd.shape)}")
        return self._pad(qd) if qd.shape[1] == self.d else qd

    def dist_sample(self, q, n_global: int, k: int) -> torch.Tensor:
        return kernels.dist_sample(self._queries(q), self.rows, n_global, k)

    def dist_tau(self, lists: torch.Tensor, k: int) -> torch.Tensor:
        return kernels.dist_tau(lists, k)

    def dist_filter(self, q, n_global: int, k: int, id_offset: int, tau: torch.Tensor) -> torch.Tensor:
        return kernels.dist_filter(self._queries(q), self.rows, n_global, k, id_offset, tau)

    def dist_filter_lists(self, q, n_global: int, k: int, id_offset: int, lists: torch.Tensor) -> torch.Tensor:
        return kernels.dist_filter_lists(self._queries(q), self.rows, n_global, k, id_offset, lists)

    # persistence (replaces faiss.write_index / read_index, trainer.py:245,257): a
    # memory-mapped bf16 shard file streamed chunk by chunk (shards.py)
    def save(self, path: str) -> None:
        shards.save_rows(self.rows if self.dp == self.d else self.rows[:, : self.d].contiguous(), path)

    @classmethod
    def load(cls, path: str, device=None) -> "FlatIPIndex":
        return cls.load_rows([path], None, None, device=device)

    @classmethod
    def load_rows(cls, paths, start=None, stop=None, device=None) -> "FlatIPIndex":
        """Rows [start, stop) of the concatenated shard files (default: all) on one device."""
        sizes, d = shards.shard_sizes(paths)
        start = 0 if start is None else int(start)
        stop = sum(sizes) if stop is None else int(stop)
        idx = cls(d, device=device, capacity=0)
        idx._buf = idx._pad(shards.load_rows(paths, start, stop, idx.device))
        idx.ntotal = stop - start
        return idx


class ShardedFlatIP:
    """Row-sharded exact IP index: one shard per rank, RCCL all-gather + device merge.

    ``local`` (the per-rank shard index), ``merge`` and ``merge_packed``
    default to the HIP implementations; they are injectable only so the
    distributed logic can be exercised with the gloo backend on CPU in tests.

    Two exchange protocols (``protocol``):

    ``"global_tau"`` (default)  every shard samples its rows, the tiny best-r
        sample lists are all-gathered so all shards agree on ONE threshold for
        the whole corpus, each shard then filters against it (collecting ~1/world
        of the candidates a standalone search would) and emits a packed top-k
        ((score key << 32) | global id, u64); one all-gather + a device merge
        gives the exact answer, certified on device (>= k candidates overall,
        no shard overflow).  An uncertified batch falls back to:
    ``"per_shard"``  exact top-k per shard (own threshold, own resolve), then
        all-gather of (scores, ids) and merge.
    """

    def __init__(self, d: int, group=None, device=None, local=None, merge=None, merge_packed=None,
                 protocol: str = "global_tau", merge_exact=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.local = local if local is not None else FlatIPIndex(d, device=device)
        self.merge = merge if merge is not None else kernels.topk_merge
        self.merge_packed = merge_packed if merge_packed is not None else kernels.merge_packed
        self.merge_exact = merge_exact if merge_exact is not None else kernels.merge_exact
        if protocol not in ("global_tau", "per_shard"):
            raise ValueError(f"unknown protocol {protocol!r}")
        self.protocol = protocol
        self.fallbacks = 0   # batches the global-tau protocol could not certify
        self.order_uncertified = 0   # queries left in the fp32 order (massive near-ties, per-shard path)
        self.d = d
        self.offset = 0      # global id of this shard's first row
        self.ntotal = 0      # rows over all shards
        self.stats = None    # GLOBAL row statistics (max over shards), set by sync_offsets
        # grouped search: run each group's exchange + merge + canonical stage on a side stream and a
        # second communicator, beside the next group's scans (_SideChannel).  Off by default: the
        # group's filter launch keeps one 153-KiB-LDS, 512-VGPR work-group on EVERY CU for its whole
        # duration, so RCCL's copy kernels only get CUs between scans either way, and the side kernels
        # then hold the next scan's work-groups back ("overlapped exchange"); the 8-GPU
        # node decides.  True: the side-stream form (tested identical on 2-3 ranks and through RCCL).
        self.overlap_exchange = False
        self._side_ch = None

    def add_shard(self, x) -> None:
        """Append rows to THIS rank's shard, then agree on the global id offsets (collective)."""
        self.local.add(x)
        self.sync_offsets()

    def sync_offsets(self):
        """Agree on the shard offsets and the corpus-wide row statistics (collective)."""
        counts = comm.all_gather_sizes(self.local.ntotal, self.local.device, self.group) if self._multi() \
            else [int(self.local.ntotal)]
        self.offset = sum(counts[: self.rank])
        self.ntotal = sum(counts)
        self.stats = None
        if isinstance(self.local, FlatIPIndex) and self.local.exact_order:
            if self.local.ntotal > 0:
                st = self.local.row_stats()
            else:   # an empty shard: the neutral element of the combination below
                st = torch.zeros(_native.ROW_STATS_LEN, dtype=torch.float32, device=self.local.device)
                st[1] = 1.0
            if self._multi():
                # max of the squared norms, AND of the integer flags (as a max of their negations)
                st = st.clone()
                st[1] = -st[1]
                comm.all_reduce_max_(st, self.group)
                st[1] = -st[1]
            self.stats = st
        return counts

    def search_device(self, q, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """Every rank passes the SAME queries; every rank gets the global top-k."""
        return self._finish(self._enqueue(q, k))

    def search_batches(self, batches, k: int):
        """search_device over a sequence of query batches (every rank passes the same batches)."""
        return list(self.search_batches_iter(batches, k))

    def search_batches_iter(self, batches, k: int, to_host: bool = False):
        """Generator form of search_batches (see FlatIPIndex.search_batches_iter).  Global-threshold
        protocol on the HIP shard: the batches run in groups of GROUP_QUERIES queries
        (_gtau_enqueue_group: one sample launch, one sample-list all-gather, one packed all-gather
        and one merge per group; one filter scan per batch), group g + 1 enqueued before the host
        checks group g's certificates.  Otherwise batch j + 1 is enqueued (scan, exchange, merge)
        before the host checks batch j's certificate."""
        batches = list(batches)
        self._check_k(k)
        if k > kernels.MAX_K:   # per batch, synchronous (the large-k path)
            for q in batches:
                r = self._search_large(q, k)
                yield (r[0].cpu().numpy(), r[1].cpu().numpy()) if to_host else r
            return
        if self._use_groups():
            groups = [[self.local._queries(q) for q in g] for g in _groups(batches)]

            def redo(q):
                if self.stats is not None:   # canonical order: exact keys per shard, merged by key (round 6)
                    return self._search_large(q, k)
                return self._finish(("pshard", q, k) + self._per_shard_enqueue(q, k))

            def fin(pend):
                res, nredo, nunc = _gtau_finish_group(pend, redo)
                self.fallbacks += nredo
                self.order_uncertified += nunc
                if nredo and getattr(self.local, "exchange_capped", True):
                    # a capped list reached into the merged top-kc (rows ordered by relevance across the
                    # shards?): every later group exchanges full lists (every rank merged the same
                    # gathered data, so every rank takes this branch)
                    self.local.exchange_capped = False
                return res

            chunks = self.group_chunks()
            if isinstance(self.local, FlatIPIndex):
                _reserve_group_memory(self.local, k, self.ntotal, chunks)
            side = self._side()
            for res in _pipeline(groups, lambda j, g: _gtau_enqueue_group(
                    self.local, g, k, self.ntotal, self.offset, self._all_gather, to_host, stats=self.stats,
                    all_reduce_sum=lambda t: comm.all_reduce_sum_(t, self.group), chunks=chunks,
                    world=self.world, side=side), fin):
                yield from res
            return
        for r in _pipeline(batches, lambda j, q: self._enqueue(q, k, to_host), self._finish):
            if to_host and isinstance(r[0], torch.Tensor):
                r = (r[0].cpu().numpy(), r[1].cpu().numpy())
            yield r

    def group_chunks(self):
        """This shard's row chunks of a group filter: as many as the largest shard needs (every rank the
        same count: the gathered part buffers have one shape; W = 8 over 10M rows: one)."""
        per = -(-self.ntotal // max(1, self.world))
        nch = len(group_chunks(per)) if GROUP_CHUNK_ROWS > 0 else 1
        return group_chunks(self.local.ntotal, nch=nch)

    def _use_groups(self) -> bool:
        """search_batches runs the grouped global-threshold protocol (one filter launch per group)."""
        return (self._multi() and self.protocol == "global_tau" and self.ntotal < 0xFFFFFFFF
                and isinstance(self.local, FlatIPIndex))

    def _all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape] all-gather (RCCL on device; host-staged under gloo, comm.py)."""
        return comm.all_gather_stacked(t, self.group)

    def _side(self):
        """The exchange side channel (_SideChannel), created on first use -- every rank runs the same
        searches, so every rank creates the second communicator at the same point.  None on a CPU shard,
        for a sub-group index (a new communicator needs every rank of the job) or with overlap_exchange
        off."""
        if not (self.overlap_exchange and self._multi() and self.local.device.type == "cuda"):
            return None
        if self.group is not None and self.group != self.dist.group.WORLD:
            return None
        if self._side_ch is None:
            xg = self.dist.new_group(ranks=list(range(self.dist.get_world_size())),
                                     backend=self.dist.get_backend())
            self._side_ch = _SideChannel(torch.cuda.Stream(self.local.device), xg)
        return self._side_ch

    def _multi(self) -> bool:
        """Exchange through collectives: world > 1 (or the test-only world-1 forcing, comm.py)."""
        return self.world > 1 or comm.collective(self.group)

    def _check_k(self, k: int):
        if k < 1 or k > kernels.MAX_K_LARGE:
            raise ValueError(f"unsupported k={k} (1 <= k <= {kernels.MAX_K_LARGE})")

    def _search_large(self, q, k: int):
        """k > 2048 (round 6; faiss answers any k, DRT/arguments.py:195 retrieve_num): every shard ranks its
        own rows canonically (exact order keys, kernels.ip_topk_exact_keys), the (key, global id) lists are
        all-gathered and merged by exact key (kernels.merge_exact) -- the single-index canonical top-k,
        since the global top-k lies in the union of the shards' top-k.  No threshold exchange, no delta
        all-reduce: the keys are exact where they are made."""
        if not self._multi():
            return self.local.search_device(q, k, id_offset=self.offset)
        keys, ids = self.local.search_exact_keys(q, k, id_offset=self.offset)
        return self.merge_exact(self._all_gather(keys.contiguous()), self._all_gather(ids.contiguous()), k)

    def _enqueue(self, q, k: int, to_host: bool = False):
        self._check_k(k)
        if k > kernels.MAX_K:
            return ("done", self._search_large(q, k))
        if not self._multi():
            if hasattr(self.local, "_enqueue"):
                return ("local", self.local._enqueue(q, k, self.offset, to_host=to_host))
            return ("done", self.local.search_device(q, k, id_offset=self.offset))
        if self.protocol == "global_tau" and self.ntotal < 0xFFFFFFFF:
            if isinstance(self.local, FlatIPIndex):
                # the HIP shard: one batch as a group of one (canonical order included)
                qd = self.local._queries(q)
                _, _, s, i, _, h, ev, _ = _gtau_enqueue_group(
                    self.local, [qd], k, self.ntotal, self.offset, self._all_gather, stats=self.stats,
                    all_reduce_sum=lambda t: comm.all_reduce_sum_(t, self.group), world=self.world)
                return ("gtau", qd, k, s, i, h, ev)
            best = self.local.dist_sample(q, self.ntotal, k)                 # [nq, r] u32 keys
            lists = self._all_gather(best)                                   # [world, nq, r]
            if hasattr(self.local, "dist_filter_lists"):                     # tau + filter fused
                packed = self.local.dist_filter_lists(q, self.ntotal, k, self.offset, lists)
            else:
                tau = self.local.dist_tau(lists, k)                          # [nq]
                packed = self.local.dist_filter(q, self.ntotal, k, self.offset, tau)   # [nq, k + 1] u64
            s, i, status = self.merge_packed(self._all_gather(packed), k, self.ntotal)
            # every rank merged the same gathered lists: the same status, the same branch
            return ("gtau", q, k, s, i) + _stage_status(status)
        return ("pshard", q, k) + self._per_shard_enqueue(q, k)

    def _per_shard_enqueue(self, q, k: int):
        if hasattr(self.local, "search_unresolved"):
            s, i, st = self.local.search_unresolved(q, k, id_offset=self.offset)
        else:   # injected test doubles return exact results
            s, i = self.local.search_device(q, k, id_offset=self.offset)
            st = torch.zeros((s.shape[0],), dtype=torch.int32, device=s.device)
        gst = self._all_gather(st)
        ms, mi = self.merge(self._all_gather(s), self._all_gather(i), k)
        # a query any rank could not certify is redone on every rank (same gathered status)
        h, ev = _stage_status(gst.amax(0))
        return ms, mi, h, ev, s, i, st

    def _finish(self, pend):
        kind = pend[0]
        if kind == "done":
            return pend[1]
        if kind == "local":
            return self.local._finish(pend[1])
        if kind == "gtau":
            _, q, k, s, i, h, ev = pend
            if _status_failed(h, ev) == 0:
                self.order_uncertified += _order_uncertified(h)
                return s, i
            self.fallbacks += 1
            if isinstance(self.local, FlatIPIndex):   # full exchange lists from now on (see search_batches_iter)
                self.local.exchange_capped = False
            if self.stats is not None:
                # canonical order (round 6): every shard's exact top-k keys merged by key -- the redo stays
                # in the fp64 order instead of merging the per-shard lists by fp32 scores
                return self._search_large(q, k)
            pend = ("pshard", q, k) + self._per_shard_enqueue(q, k)
        _, q, k, ms, mi, h, ev, s, i, st = pend
        if _status_failed(h, ev) == 0:
            return ms, mi
        # some rank has uncertified queries: each rank redoes its own exactly, then re-merge
        nres = kernels.resolve_failed(self.local._queries(q), self.local.rows, k, self.offset, s, i, st)
        self.local.resolved += nres
        return self.merge(self._all_gather(s), self._all_gather(i), k)

    def search(self, q, k: int) -> Tuple[np.ndarray, np.ndarray]:
        s, i = self.search_device(q, k)
        return s.cpu().numpy(), i.cpu().numpy()

    # persistence: every rank writes its own shard file; any world size reads them back
    def save_shard(self, directory: str, ep) -> str:
        """Write THIS rank's rows to ``{ep}.{rank}.bf16.npy`` (replaces trainer.py:210-216)."""
        import os
        os.makedirs(directory, exist_ok=True)
        path = shards.shard_path(directory, ep, self.rank)
        self.local.save(path)
        return path

    @classmethod
    def load_shards(cls, directory: str, ep, group=None, device=None, **kw) -> "ShardedFlatIP":
        """Each rank maps the shard files of ``ep`` (in rank order) and streams its contiguous
        global row range into HBM; the files may come from a different world size.
        Replaces the rank-0 index build + every-rank index read (trainer.py:220-262)."""
        paths = shards.list_shards(directory, ep)
        sizes, d = shards.shard_sizes(paths)
        self = cls(d, group=group, device=device, **kw)
        a, b = shards.split_rows(sum(sizes), self.world, self.rank)
        if kw.get("local") is None:
            self.local = FlatIPIndex.load_rows(paths, a, b, device=self.local.device)
        else:
            self.local.add(shards.load_rows(paths, a, b, torch.device("cpu")).float())
        self.sync_offsets()
        return self
