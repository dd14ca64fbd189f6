"""Drop-in for DRT/model/reranker.py (RRModel, RROutput): cross-encoder reranking.

``RRModel.encode`` (reranker.py:111-130): pair forward ([CLS] q [SEP] d [SEP],
L = q_max_len + p_max_len = 160) -> pooling -> LinearHead(768 -> 1) score.  When
no gradient can be asked for (grad mode off or a frozen tower) the whole pair
tower runs on the HIP inference kernels (the same bf16 MFMA GEMMs + fused
attention as the bi-encoder) and the 768 -> 1 head on the HIP GEMM; with grad on
(training, or eval mode with grad) BERT pair towers up to L = 512 run on the HIP
training tower (model/train_tower.py, forward + backward on HIP kernels, HF
train-mode dropout), other towers on the HF module under autograd.  T5
rerankers (logits of pos/neg tokens, :115-119) are outside the MI355X path.
"""
from __future__ import annotations

import json
import logging
import os
from dataclasses import dataclass
from typing import Dict

import torch
import torch.nn as nn
from torch import Tensor
from transformers import AutoConfig, AutoModel, BatchEncoding, PreTrainedModel
from transformers.modeling_outputs import ModelOutput

from ..trainer.losses import CrossEntropyLoss, rr_loss_functions
from .encoder import HipBertEncoder, linear_head
from .linear import LinearHead
from .train_tower import MAX_TRAIN_SEQ, tower_supported, train_hidden

logger = logging.getLogger(__name__)


@dataclass
class RROutput(ModelOutput):
    pos_pair_scores: Tensor = None
    neg_pair_scores: Tensor = None
    loss: Tensor = None


class RRModel(nn.Module):
    def __init__(self, lm: PreTrainedModel, head: nn.Module, feature: str = "last_hidden_state",
                 pooling: str = "first", pos_token: str = None, neg_token: str = None, tokenizer=None,
                 model_args=None, data_args=None, train_args=None):
        super().__init__()
        self.lm = lm
        self.head = head
        self.feature = feature
        self.pooling = pooling
        self.pos_token = pos_token
        self.neg_token = neg_token
        self.tokenizer = tokenizer
        self.pos_token_id = tokenizer.encode(pos_token, add_special_tokens=False)[0] if pos_token else None
        self.neg_token_id = tokenizer.encode(neg_token, add_special_tokens=False)[0] if neg_token else None
        self.model_args = model_args
        self.data_args = data_args
        self.train_args = train_args
        self._hip = None
        if train_args is not None:
            self.loss_fn_str = train_args.loss_fn
            self.margin = train_args.margin
            self.loss_fn = rr_loss_functions[self.loss_fn_str](self.margin)
        if "T5" in type(self.lm).__name__ and not getattr(model_args, "encoder_only", False):
            self.loss_fn_str = "ce"
            self.loss_fn = CrossEntropyLoss()

    def _get_config_dict(self):
        return {"plm_backbone": {"type": type(self.lm).__name__, "feature": self.feature},
                "pooling": self.pooling, "pos_token": self.pos_token, "neg_token": self.neg_token}

    def forward(self, pos_pairs: Dict[str, Tensor] = None, neg_pairs: Dict[str, Tensor] = None):
        pos = self.encode(pos_pairs)
        if neg_pairs is None:
            return pos
        neg = self.encode(neg_pairs)
        if pos.shape != neg.shape:
            return RROutput(pos_pair_scores=pos, neg_pair_scores=neg)
        return RROutput(loss=self.loss_fn(pos, neg), pos_pair_scores=pos, neg_pair_scores=neg)

    def _hip_state(self):
        dev = next(self.lm.parameters()).device
        ver = tuple(p._version for p in self.lm.parameters()) + (self.head.linear.weight._version, str(dev))
        if self._hip is None or self._hip[0] != ver:
            if type(self.lm).__name__ != "BertModel":
                raise NotImplementedError(f"HIP reranker supports BERT-family towers only (got {type(self.lm).__name__})")
            enc = HipBertEncoder.from_hf(self.lm, dev)
            w = self.head.linear.weight.detach().to(torch.bfloat16).contiguous()
            self._hip = (ver, enc, w)
        return self._hip[1], self._hip[2]

    def encode(self, items):
        if items is None:
            return None, None
        items = BatchEncoding(items)
        if "T5" in type(self.lm).__name__ and not getattr(self.model_args, "encoder_only", False):
            raise NotImplementedError("T5 rerankers are outside the MI355X hot path")
        if self.pooling not in ("first", "mean"):
            raise ValueError("Unknown pooling type: {}".format(self.pooling))
        dev = next(self.lm.parameters()).device
        # inference kernels only when no gradient can be asked for (grad mode off or a frozen
        # tower); eval mode with grad on returns differentiable scores as the reference does
        frozen = not any(p.requires_grad for p in self.lm.parameters())
        if dev.type == "cuda" and (not torch.is_grad_enabled() or frozen):
            enc, w = self._hip_state()
            mask = items.get("attention_mask")
            hidden = enc(items["input_ids"], mask, items.get("token_type_ids"))
            _, rb = enc.pool(hidden, mask, self.pooling, want_bf16=True)
            return linear_head(rb, w)  # [B, 1] fp32
        if (dev.type == "cuda" and self.feature == "last_hidden_state"
                and tower_supported(self.lm) is None and items["input_ids"].shape[1] <= MAX_TRAIN_SEQ):
            # pair forward + backward on the HIP training tower (model/train_tower.py)
            hidden = train_hidden(self.lm, items["input_ids"], items.get("attention_mask"),
                                  token_type_ids=items.get("token_type_ids"))
        else:
            from .biencoder import _log_fallback
            _log_fallback("reranker: " + ("tower on the CPU" if dev.type != "cuda" else
                                          tower_supported(self.lm) or "feature / length"))
            out = self.lm(**items, return_dict=True)
            hidden = getattr(out, self.feature)
        if self.pooling == "first":
            reps = hidden[:, 0, :]
        else:
            m = items.attention_mask.unsqueeze(-1).expand(hidden.size()).float()
            reps = torch.sum(hidden * m, 1) / torch.clamp(m.sum(1), min=1e-9)
        return self.head(reps)

    @classmethod
    def build(cls, model_args, data_args=None, train_args=None, tokenizer=None, **hf_kwargs):
        from transformers import T5EncoderModel, T5ForConditionalGeneration
        config = None
        hf_config = AutoConfig.from_pretrained(model_args.model_name_or_path, **hf_kwargs)
        if getattr(model_args, "encoder_only", False):
            model_class = T5EncoderModel
        elif "T5" in hf_config.architectures[0]:
            model_class = T5ForConditionalGeneration
        else:
            model_class = AutoModel
        cfg = os.path.join(model_args.model_name_or_path, "openmatch_config.json")
        if os.path.exists(cfg):
            with open(cfg) as f:
                config = json.load(f)
        if os.path.isdir(model_args.model_name_or_path) and config is not None:
            lm = model_class.from_pretrained(model_args.model_name_or_path, **hf_kwargs)
            head = LinearHead.load(ckpt_dir=model_args.model_name_or_path)
        else:
            lm = model_class.from_pretrained(model_args.model_name_or_path, **hf_kwargs)
            head = LinearHead(model_args.projection_in_dim, 1)
        return cls(lm=lm, head=head,
                   feature=model_args.feature if config is None else config["plm_backbone"]["feature"],
                   pooling=model_args.pooling if config is None else config["pooling"],
                   pos_token=model_args.pos_token if config is None else config["pos_token"],
                   neg_token=model_args.neg_token if config is None else config["neg_token"],
                   tokenizer=tokenizer, model_args=model_args, data_args=data_args, train_args=train_args)

    def save(self, output_dir: str):
        self.lm.save_pretrained(output_dir)
        self.head.save(output_dir)
        with open(os.path.join(output_dir, "openmatch_config.json"), "w") as f:
            json.dump(self._get_config_dict(), f, indent=4)
