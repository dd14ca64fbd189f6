"""Drop-in for DRT/model/biencoder.py (DRModel, DRModelForInference, DROutput).

Same constructor, ``build``/``save``/``load``/``encode``/``forward`` contract
and checkpoint format (HF ``save_pretrained`` per tower + ``openmatch_config.json``,
biencoder.py:159-241).  What changes is where the arithmetic runs:

* encode without autograd (grad mode off or a frozen tower — Trainer.evaluate /
  _encoding_corpus, DRModelForInference) runs the whole tower on the HIP inference
  kernels (model/encoder.HipBertEncoder): bf16 MFMA GEMMs, fused attention, fp32
  LayerNorm statistics, pooling / head / L2-normalise kernels.  ``hidden`` is
  returned in bf16, ``reps`` in fp32.
* encode with autograd (training, or eval mode with grad on, where the reference
  returns differentiable reps) runs BERT towers up to L = 512 on the HIP training
  tower (model/train_tower.py: forward with saved bf16 activations + backward on
  HIP kernels, HF train-mode dropout regenerated from a counter hash; dropout is
  off in eval mode); other towers stay on the HF module under autograd.
* the training score matrix + cross entropy (forward :107-119) runs on the
  fused fp32 kernels with autograd (torch.ops.drt.score_ce_fwd, score_ce.py).
"""
from __future__ import annotations

import copy
import json
import logging
import os
from dataclasses import dataclass
from typing import Dict, Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F
from torch import Tensor
from transformers import AutoModel, BatchEncoding, PreTrainedModel
from transformers.modeling_outputs import ModelOutput

from .encoder import HipBertEncoder, l2_normalize_, linear_head
from .train_tower import MAX_TRAIN_SEQ, tower_supported, train_hidden
from .linear import LinearHead

logger = logging.getLogger(__name__)


@dataclass
class DROutput(ModelOutput):
    q_reps: Tensor = None
    p_reps: Tensor = None
    loss: Tensor = None
    scores: Tensor = None


_FALLBACK_LOGGED = set()


def _log_fallback(why: str):
    """Once per reason: an encode that cannot take the HIP towers runs the HF module under torch
    (the reference's own arithmetic) -- say so instead of silently."""
    if why not in _FALLBACK_LOGGED:
        _FALLBACK_LOGGED.add(why)
        logger.warning("DRModel.encode: HF module under torch, not the HIP tower (%s)", why)


def _torch_mean_pooling(h, mask):
    m = mask.unsqueeze(-1).expand(h.size()).float()
    return torch.sum(h * m, 1) / torch.clamp(m.sum(1), min=1e-9)


def _torch_max_pooling(h, mask):
    m = mask.unsqueeze(-1).expand(h.size()).float()
    return torch.max(h * m, 1)[0]


class DRModel(nn.Module):
    def __init__(self, lm_q: PreTrainedModel, lm_p: PreTrainedModel, tied: bool = True,
                 feature: str = "last_hidden_state", pooling: str = "first", head_q: nn.Module = None,
                 head_p: nn.Module = None, normalize: bool = False, model_args=None, data_args=None,
                 train_args=None):
        super().__init__()
        self.tied = tied
        self.lm_q = lm_q
        self.lm_p = lm_p
        self.head_q = head_q
        self.head_p = head_p
        self.loss_fn = nn.CrossEntropyLoss(reduction="mean")
        self.feature = feature
        self.pooling = pooling
        self.hip_train = True   # HIP training tower for BERT towers with L <= 512 (set False: HF autograd)
        self.normalize = normalize
        self.model_args = model_args
        self.train_args = train_args
        self.data_args = data_args
        self._hip_cache: Dict[int, tuple] = {}
        if train_args is not None and getattr(train_args, "negatives_x_device", False):
            if not dist.is_initialized():
                raise ValueError("Distributed training has not been initialized for representation all gather.")
            self.process_rank = dist.get_rank()
            self.world_size = dist.get_world_size()

    def _get_config_dict(self):
        return {
            "tied": self.tied,
            "plm_backbone": {"type": type(self.lm_q).__name__, "feature": self.feature},
            "pooling": self.pooling,
            "linear_head": bool(self.head_q),
            "normalize": self.normalize,
        }

    # ------------------------------------------------------------------
    def forward(self, query: Dict[str, Tensor] = None, passage: Dict[str, Tensor] = None):
        q_hidden, q_reps = self.encode_query(query)
        p_hidden, p_reps = self.encode_passage(passage)
        if query is None or passage is None:
            return DROutput(q_reps=q_reps, p_reps=p_reps)
        x_dev = bool(self.train_args is not None and getattr(self.train_args, "negatives_x_device", False))
        if x_dev:
            q_reps = self.dist_gather_tensor(q_reps)
            p_reps = self.dist_gather_tensor(p_reps)
        n_passages = self.data_args.train_n_passages
        scale = float(self.world_size) if (self.training and x_dev) else 1.0
        from ..score_ce import score_ce
        if q_reps.is_cuda:
            loss, scores = score_ce(q_reps, p_reps, n_passages, scale)
        elif torch.cuda.is_available():
            # a tower on the CPU (the reference scores on any device, biencoder.py:107-116): the reps go to
            # the GPU for the fused HIP op and the loss / scores come back; autograd carries the gradients
            # across both copies to the CPU tower
            dev = torch.device("cuda", torch.cuda.current_device())
            loss, scores = score_ce(q_reps.to(dev), p_reps.to(dev), n_passages, scale)
            loss, scores = loss.to(q_reps.device), scores.to(q_reps.device)
        else:
            raise ValueError("DRModel.forward: the MI355X build computes the score matrix on the GPU only "
                             "(no GPU visible)")
        return DROutput(loss=loss, scores=scores, q_reps=q_reps, p_reps=p_reps)

    # ------------------------------------------------------------------
    def _hip_encoder(self, model) -> HipBertEncoder:
        dev = next(model.parameters()).device
        key = id(model)
        ver = tuple(p._version for p in model.parameters()) + (str(dev),)
        hit = self._hip_cache.get(key)
        if hit is None or hit[0] != ver:
            if type(model).__name__ not in ("BertModel",):
                raise NotImplementedError(
                    f"HIP encoder supports BERT-family towers only (got {type(model).__name__})")
            enc = HipBertEncoder.from_hf(model, dev)
            self._hip_cache[key] = (ver, enc)
            return enc
        return hit[1]

    def _head_weight(self, head) -> torch.Tensor:
        w = head.linear.weight
        key = id(head)
        ver = (w._version, str(w.device))
        hit = self._hip_cache.get(key)
        if hit is None or hit[0] != ver:
            wb = w.detach().to(torch.bfloat16).contiguous()
            self._hip_cache[key] = (ver, wb)
            return wb
        return hit[1]

    def _use_hip(self, model) -> bool:
        """Inference kernels (no autograd) when no gradient can be asked for: grad mode off, or
        a frozen tower.  Eval mode with grad on (the reference returns differentiable reps
        there) takes the training tower, which drops dropout when the module is in eval."""
        dev = next(model.parameters()).device
        if dev.type != "cuda":
            return False
        return not torch.is_grad_enabled() or not any(p.requires_grad for p in model.parameters())

    def encode(self, items, model, head):
        if items is None:
            return None, None
        items = BatchEncoding(items)
        if "T5" in type(model).__name__ and not getattr(self.model_args, "encoder_only", False):
            raise NotImplementedError("T5 towers are outside the MI355X hot path (BERT-family encoders only)")
        if self.pooling not in ("first", "mean", "max"):
            raise ValueError("Unknown pooling type: {}".format(self.pooling))
        # a feature other than last_hidden_state (arguments.py:34-37) is off the HIP path in both modes:
        # it takes the HF module below, with the reason logged, whether or not autograd is on
        if self._use_hip(model) and self.feature == "last_hidden_state":
            enc = self._hip_encoder(model)
            hidden = enc(items["input_ids"], items.get("attention_mask"), items.get("token_type_ids"))
            reps, rb = enc.pool(hidden, items.get("attention_mask"), self.pooling, want_bf16=head is not None)
            if head is not None:
                reps = linear_head(rb, self._head_weight(head))
            if self.normalize:
                reps, _ = l2_normalize_(reps)
            return hidden, reps
        # forward with autograd: BERT towers up to MAX_TRAIN_SEQ tokens run the HIP training tower
        # (saved bf16 activations + backward on HIP kernels, HF dropout semantics in train mode,
        # model/train_tower.py); anything else keeps the HF module under autograd.
        why = None
        if self.feature != "last_hidden_state":
            why = f"feature {self.feature!r}"
        elif not self.hip_train:
            why = "hip_train = False"
        elif not next(model.parameters()).is_cuda:
            why = "tower on the CPU"
        elif items["input_ids"].shape[1] > MAX_TRAIN_SEQ:
            why = f"sequence length {items['input_ids'].shape[1]} > {MAX_TRAIN_SEQ}"
        else:
            why = tower_supported(model)
        if why is None:
            hidden = train_hidden(model, items["input_ids"], items.get("attention_mask"),
                                  token_type_ids=items.get("token_type_ids"))
        else:
            _log_fallback(why)
            out = model(**items, return_dict=True)
            hidden = getattr(out, self.feature)
        if self.pooling == "first":
            reps = hidden[:, 0, :]
        elif self.pooling == "mean":
            reps = _torch_mean_pooling(hidden, items.attention_mask)
        else:
            reps = _torch_max_pooling(hidden, items.attention_mask)
        if head is not None:
            reps = head(reps)
        if self.normalize:
            reps = F.normalize(reps, dim=1)
        return hidden, reps

    def encode_passage(self, psg):
        return self.encode(psg, self.lm_p, self.head_p)

    def encode_query(self, qry):
        return self.encode(qry, self.lm_q, self.head_q)

    # ------------------------------------------------------------------
    @classmethod
    def build(cls, model_args, data_args=None, train_args=None, **hf_kwargs):
        from transformers import T5EncoderModel
        config = None
        model_class = T5EncoderModel if getattr(model_args, "encoder_only", False) else AutoModel
        head_q = head_p = None
        cfg_path = os.path.join(model_args.model_name_or_path, "openmatch_config.json")
        if os.path.exists(cfg_path):
            with open(cfg_path) as f:
                config = json.load(f)
        if os.path.isdir(model_args.model_name_or_path) and config is not None:
            tied = config["tied"]
            if tied:
                lm_q = lm_p = model_class.from_pretrained(model_args.model_name_or_path, **hf_kwargs)
                if config["linear_head"]:
                    head_q = head_p = LinearHead.load(model_args.model_name_or_path)
            else:
                root = model_args.model_name_or_path
                lm_q = model_class.from_pretrained(os.path.join(root, "query_model"), **hf_kwargs)
                lm_p = model_class.from_pretrained(os.path.join(root, "passage_model"), **hf_kwargs)
                if config["linear_head"]:
                    head_q = LinearHead.load(os.path.join(root, "query_head"))
                    head_p = LinearHead.load(os.path.join(root, "passage_head"))
        else:
            tied = not model_args.untie_encoder
            lm_q = model_class.from_pretrained(model_args.model_name_or_path, **hf_kwargs)
            lm_p = copy.deepcopy(lm_q) if not tied else lm_q
            if model_args.add_linear_head:
                head_q = LinearHead(model_args.projection_in_dim, model_args.projection_out_dim)
                head_p = copy.deepcopy(head_q) if not tied else head_q
        return cls(
            lm_q=lm_q, lm_p=lm_p, tied=tied,
            feature=model_args.feature if config is None else config["plm_backbone"]["feature"],
            pooling=model_args.pooling if config is None else config["pooling"],
            head_q=head_q, head_p=head_p,
            normalize=model_args.normalize if config is None else config["normalize"],
            model_args=model_args, data_args=data_args, train_args=train_args,
        )

    def save(self, output_dir: str):
        if not self.tied:
            os.makedirs(os.path.join(output_dir, "query_model"), exist_ok=True)
            os.makedirs(os.path.join(output_dir, "passage_model"), exist_ok=True)
            self.lm_q.save_pretrained(os.path.join(output_dir, "query_model"))
            self.lm_p.save_pretrained(os.path.join(output_dir, "passage_model"))
            if self.head_q is not None:
                os.makedirs(os.path.join(output_dir, "query_head"), exist_ok=True)
                os.makedirs(os.path.join(output_dir, "passage_head"), exist_ok=True)
                self.head_q.save(os.path.join(output_dir, "query_head"))
                self.head_p.save(os.path.join(output_dir, "passage_head"))
        else:
            self.lm_q.save_pretrained(output_dir)
            if self.head_q is not None:
                self.head_q.save(output_dir)
        with open(os.path.join(output_dir, "openmatch_config.json"), "w") as f:
            json.dump(self._get_config_dict(), f, indent=4)

    def dist_gather_tensor(self, t: Optional[torch.Tensor]):
        if t is None:
            return None
        # same semantics as the reference (biencoder.py:243-254): the other ranks' slices are
        # detached copies, this rank's slice is `t` itself so its gradient flows back
        from .. import comm
        t = t.contiguous()
        all_tensors = comm.all_gather_list(t)
        all_tensors[self.process_rank] = t
        return torch.cat(all_tensors, dim=0)

    def get_model_ckpt(self):
        return self.lm_q.state_dict()

    def load(self, _state_dict):
        self.lm_q.load_state_dict(_state_dict)
        self.lm_p.load_state_dict(_state_dict)


class DRModelForInference(DRModel):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)

    @torch.no_grad()
    def encode_passage(self, psg):
        return super().encode_passage(psg)

    @torch.no_grad()
    def encode_query(self, qry):
        return super().encode_query(qry)

    def forward(self, query: Dict[str, Tensor] = None, passage: Dict[str, Tensor] = None):
        q_hidden, q_reps = self.encode_query(query)
        p_hidden, p_reps = self.encode_passage(passage)
        return DROutput(q_reps=q_reps, p_reps=p_reps)
