"""Collectives of the hot path, one place for the backend rules.

On the production backend (``nccl`` = RCCL on ROCm, over xGMI) device tensors go
straight into the collective.  Under ``gloo`` (the multi-rank CPU tests, and
several ranks rehearsing the N > 1 protocol on ONE shared GPU) gloo cannot take
HIP tensors for all-gather, so the payload is staged through host memory and
the result is moved back to the caller's device.  The data path is otherwise
identical, which is what lets the shared-GPU tests exercise the real kernels.

Reference collectives replaced / kept: ``dist.all_gather`` of reps
(DRT/model/biencoder.py:243-254, DRT/trainer/losses.py:38); the file-system
exchange of corpus embeddings (DRT/trainer/trainer.py:210-262) becomes an
all-gather of per-shard top-k lists (search.ShardedFlatIP).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


def world_rank(group=None):
    if not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


# Test-only switch: take the collective code path even in a world-1 group, so a one-GPU box
# drives the device-tensor branch of every collective below through a real RCCL communicator
# (tests/test_rccl_gpu.py).  Production never sets it: a world-1 collective is a copy.
_FORCE = False


def force_collectives(on: bool) -> None:
    global _FORCE
    _FORCE = bool(on)


def collective(group=None) -> bool:
    """True when a call must go through torch.distributed: world > 1, or forced at world 1."""
    if not dist.is_initialized():
        return False
    return _FORCE or dist.get_world_size(group) > 1


def is_gloo(group=None) -> bool:
    return dist.is_initialized() and dist.get_backend(group) == "gloo"


def comm_device(t: torch.Tensor, group=None) -> torch.device:
    """Where the collective's buffers live: host for gloo, the tensor's device otherwise."""
    return torch.device("cpu") if is_gloo(group) else t.device


def all_gather_stacked(t: torch.Tensor, group=None) -> torch.Tensor:
    """[world, *t.shape] on t.device: every rank's (same-shaped) tensor, in rank order."""
    world, _ = world_rank(group)
    if not collective(group):
        return t.unsqueeze(0)
    cd = comm_device(t, group)
    src = t.detach().contiguous().to(cd)
    out = torch.empty((world * src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=cd)
    dist.all_gather_into_tensor(out, src, group=group)
    return out.to(t.device).view((world,) + tuple(t.shape))


def all_gather_list(t: torch.Tensor, group=None) -> List[torch.Tensor]:
    """Per-rank list of detached copies (the reference's ``dist.all_gather`` into ``empty_like``)."""
    return list(all_gather_stacked(t, group).unbind(0))


def all_gather_sizes(n: int, device: Optional[torch.device] = None, group=None) -> List[int]:
    if not collective(group):
        return [int(n)]
    dev = torch.device("cpu") if is_gloo(group) or device is None else device
    v = torch.tensor([int(n)], dtype=torch.int64, device=dev)
    return [int(x) for x in all_gather_stacked(v, group).view(-1).tolist()]


def all_gather_rows(t: torch.Tensor, group=None):
    """Variable-length row concatenation: returns (rows of every rank concatenated, sizes).
    Rows are padded to the largest rank's count for the collective and the padding dropped."""
    world, _ = world_rank(group)
    sizes = all_gather_sizes(t.shape[0], t.device, group)
    if not collective(group):
        return t, sizes
    mx = max(sizes)
    pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    allp = all_gather_stacked(pad, group)
    return torch.cat([allp[r, : sizes[r]] for r in range(world)], 0), sizes


def all_reduce_max_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place MAX all-reduce (staged through host under gloo)."""
    if not collective(group):
        return t
    if is_gloo(group) and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MAX, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t


def all_reduce_sum_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place SUM all-reduce (staged through host under gloo)."""
    if not collective(group):
        return t
    if is_gloo(group) and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t
