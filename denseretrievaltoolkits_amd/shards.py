"""Corpus-embedding shard files: memory-mapped bf16 rows streamed to/from HBM.

Replaces the reference's corpus round trip:
  * ``Trainer._encoding_corpus`` writes ``{ep}.{rank}.npy`` fp32 plus a JSON id list
    (DRT/trainer/trainer.py:210-216);
  * ``Trainer._index_corpus`` has rank 0 ``np.load`` every rank file in ``os.listdir``
    order into one faiss index and write it out; every rank then reads the whole
    index back (trainer.py:223-248, 252-261; retrieval.py:45-53 concatenates shards
    the same way) — O(N·d·W) host memory and a row order set by the filesystem.

Here a shard file is a standard ``.npy`` of int16 ``[n, d]`` holding the bf16 bit
patterns of the rows (numpy has no bf16), so ``np.load(mmap_mode="r")`` maps it
without reading it.  Files are ordered by their rank number, never by directory
listing.  Saving streams device → pinned host chunk → mapped file, loading
streams mapped file → pinned chunk → device, so neither side ever holds more
than one chunk of a shard in host memory.  A set of files written by W ranks
can be loaded by any number of ranks: rank r takes the contiguous global rows
``[r·⌈N/W'⌉, min(N, (r+1)·⌈N/W'⌉))`` (the same split as ``ShardedFlatIP``), read
across file boundaries.
"""
from __future__ import annotations

import os
import re
from typing import List, Sequence, Tuple

import numpy as np
import torch

DEFAULT_CHUNK_BYTES = 64 << 20


def shard_path(directory: str, ep, rank: int) -> str:
    return os.path.join(directory, f"{ep}.{rank}.bf16.npy")


def list_shards(directory: str, ep) -> List[str]:
    """The shard files of epoch ``ep`` ordered by rank (0, 1, ...); a gap is an error."""
    pat = re.compile(rf"^{re.escape(str(ep))}\.(\d+)\.bf16\.npy$")
    found = {}
    for name in os.listdir(directory):
        m = pat.match(name)
        if m:
            found[int(m.group(1))] = os.path.join(directory, name)
    if not found:
        raise FileNotFoundError(f"no shard files {ep}.<rank>.bf16.npy in {directory}")
    ranks = sorted(found)
    if ranks != list(range(len(ranks))):
        raise FileNotFoundError(f"shard files of epoch {ep} in {directory} are not ranks 0..{len(ranks) - 1}: {ranks}")
    return [found[r] for r in ranks]


def _chunk_rows(d: int, chunk_bytes: int) -> int:
    return max(1, chunk_bytes // (2 * d))


def save_rows(rows: torch.Tensor, path: str, chunk_bytes: int = DEFAULT_CHUNK_BYTES) -> None:
    """Write bf16 rows ``[n, d]`` (any device) to ``path`` as a mapped int16 ``.npy``."""
    if rows.dim() != 2 or rows.dtype != torch.bfloat16:
        raise ValueError(f"save_rows: expected bf16 [n, d], got {rows.dtype} {tuple(rows.shape)}")
    n, d = rows.shape
    out = np.lib.format.open_memmap(path, mode="w+", dtype=np.int16, shape=(n, d))
    step = _chunk_rows(d, chunk_bytes)
    pin = rows.is_cuda
    host = torch.empty((min(step, max(n, 1)), d), dtype=torch.int16, pin_memory=pin)
    src = rows.view(torch.int16)
    for a in range(0, n, step):
        b = min(n, a + step)
        h = host[: b - a]
        h.copy_(src[a:b], non_blocking=False)
        out[a:b] = h.numpy()
    out.flush()
    del out


def shard_sizes(paths: Sequence[str]) -> Tuple[List[int], int]:
    """Row counts of the files (header reads only) and their common dimension."""
    sizes, dim = [], None
    for p in paths:
        mm = np.load(p, mmap_mode="r", allow_pickle=False)
        if mm.ndim != 2 or mm.dtype != np.int16:
            raise ValueError(f"{p}: not a bf16 shard file (int16 [n, d]), got {mm.dtype} {mm.shape}")
        if dim is None:
            dim = int(mm.shape[1])
        elif int(mm.shape[1]) != dim:
            raise ValueError(f"{p}: dimension {mm.shape[1]} != {dim}")
        sizes.append(int(mm.shape[0]))
    return sizes, int(dim or 0)


def split_rows(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Rank ``rank``'s contiguous global row range: ceil split, no padding or duplicates."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    per = -(-n_total // world) if n_total else 0
    a = min(n_total, rank * per)
    return a, min(n_total, a + per)


def plan_reads(sizes: Sequence[int], start: int, stop: int) -> List[Tuple[int, int, int]]:
    """(file index, first row, last row + 1) pieces covering global rows [start, stop)."""
    pieces, base = [], 0
    for f, n in enumerate(sizes):
        a, b = max(start, base), min(stop, base + n)
        if a < b:
            pieces.append((f, a - base, b - base))
        base += n
    if stop > base:
        raise ValueError(f"rows [{start}, {stop}) exceed the {base} rows of the shard files")
    return pieces


def load_rows(paths: Sequence[str], start: int, stop: int, device,
              chunk_bytes: int = DEFAULT_CHUNK_BYTES) -> torch.Tensor:
    """Global rows [start, stop) of the concatenated shard files as a bf16 tensor on ``device``."""
    sizes, d = shard_sizes(paths)
    device = torch.device(device)
    out = torch.empty((stop - start, d), dtype=torch.bfloat16, device=device)
    dst = out.view(torch.int16)
    step = _chunk_rows(d, chunk_bytes)
    pin = device.type == "cuda"
    # two pinned staging buffers: the H2D copy of one overlaps the page-in of the other
    bufs = [torch.empty((max(1, min(step, stop - start)), d), dtype=torch.int16, pin_memory=pin) for _ in range(2)]
    done = [None, None]
    o, slot = 0, 0
    for f, a, b in plan_reads(sizes, start, stop):
        mm = np.load(paths[f], mmap_mode="r", allow_pickle=False)
        for c in range(a, b, step):
            e = min(b, c + step)
            if done[slot] is not None:
                done[slot].synchronize()   # the copy that last read this buffer has finished
            h = bufs[slot][: e - c]
            h.numpy()[:] = mm[c:e]
            dst[o: o + (e - c)].copy_(h, non_blocking=pin)
            if pin:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(device))
                done[slot] = ev
            o += e - c
            slot ^= 1
        del mm
    if pin:
        torch.cuda.current_stream(device).synchronize()
    return out
