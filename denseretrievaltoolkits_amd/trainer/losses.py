"""Contrastive losses with the reference's API (DRT/trainer/losses.py:7-45); the
score matrix + cross entropy runs on the fused fp32 HIP op (torch.ops.drt.score_ce_fwd, score_ce.py).
The reranker losses (:48-88) are elementwise torch and kept as is in spirit."""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import Tensor, nn

from ..score_ce import score_ce


class SimpleContrastiveLoss(nn.Module):
    def forward(self, x: Tensor, y: Tensor, target: Tensor = None, reduction: str = "mean"):
        if target is not None or reduction != "mean":
            # arbitrary targets / reductions: plain logits + torch CE (not the hot path)
            if target is None:
                per = y.size(0) // x.size(0)
                target = torch.arange(0, x.size(0) * per, per, device=x.device, dtype=torch.long)
            logits = torch.matmul(x, y.transpose(0, 1))
            return F.cross_entropy(logits, target, reduction=reduction)
        loss, _ = score_ce(x, y, y.size(0) // x.size(0), 1.0)
        return loss


class DistributedContrastiveLoss(SimpleContrastiveLoss):
    def __init__(self, n_target: int = 0, scale_loss: bool = True):
        assert dist.is_initialized(), "Distributed training has not been properly initialized."
        super().__init__()
        self.word_size = dist.get_world_size()
        self.rank = dist.get_rank()
        self.scale_loss = scale_loss

    def forward(self, x: Tensor, y: Tensor, **kwargs):
        dx, dy = self.gather_tensor(x), self.gather_tensor(y)
        loss = super().forward(dx, dy, **kwargs)
        return loss * self.word_size if self.scale_loss else loss

    def gather_tensor(self, t):
        from .. import comm
        gathered = comm.all_gather_list(t.contiguous())
        gathered[self.rank] = t
        return torch.cat(gathered, dim=0)


def get_loss_function(training_args):
    if training_args.loss_fn == "SimpleContrastiveLoss":
        return DistributedContrastiveLoss() if dist.is_initialized() else SimpleContrastiveLoss()
    return None


class MarginRankingLoss:
    def __init__(self, margin: float = 1.0):
        self.margin = margin

    def __call__(self, pos_scores, neg_scores):
        return torch.mean(F.relu(self.margin - pos_scores + neg_scores))


class SoftMarginRankingLoss:
    def __init__(self, margin: float = 1.0):
        self.margin = margin

    def __call__(self, pos_scores, neg_scores):
        return torch.mean(F.softplus(self.margin - pos_scores + neg_scores))


class BinaryCrossEntropyLoss:
    def __init__(self, margin: float = 1.0):
        pass

    def __call__(self, pos_scores, neg_scores):
        return (F.binary_cross_entropy_with_logits(pos_scores, torch.ones_like(pos_scores))
                + F.binary_cross_entropy_with_logits(neg_scores, torch.zeros_like(neg_scores)))


class CrossEntropyLoss:
    def __init__(self, margin: float = 1.0):
        pass

    def __call__(self, pos_scores, neg_scores):
        ones = torch.ones(pos_scores.shape[0], dtype=torch.long, device=pos_scores.device)
        zeros = torch.zeros(neg_scores.shape[0], dtype=torch.long, device=pos_scores.device)
        return F.cross_entropy(pos_scores, ones) + F.cross_entropy(neg_scores, zeros)


rr_loss_functions = {"mr": MarginRankingLoss, "smr": SoftMarginRankingLoss, "bce": BinaryCrossEntropyLoss,
                     "ce": CrossEntropyLoss}
