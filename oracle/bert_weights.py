"""Deterministic BERT weights + synthetic token batches — TEST INFRASTRUCTURE ONLY.

No checkpoint can be fetched offline, so parity runs use weights
that are a pure function of (seed, parameter name, shape): numpy PCG64 seeded
with (seed, crc32(name)).  Linear / embedding weights ~ N(0, 0.02) (HF's
initializer_range), biases ~ N(0, 0.02), LayerNorm gamma ~ 1 + N(0, 0.05),
beta ~ N(0, 0.05) (non-trivial so LayerNorm parameters are exercised).
Token batches follow the collator format (DRT/dataset/data_collator.py:6-15):
[CLS]=101 ... [SEP]=102, right-padded with 0, no token_type_ids.
"""
from __future__ import annotations

import zlib

import numpy as np


def bert_config(layers=12, hidden=768, heads=12, intermediate=3072, vocab=30522, max_pos=512):
    from transformers import BertConfig
    return BertConfig(vocab_size=vocab, hidden_size=hidden, num_hidden_layers=layers, num_attention_heads=heads,
                      intermediate_size=intermediate, max_position_embeddings=max_pos,
                      hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)


def param_value(seed: int, name: str, shape) -> np.ndarray:
    rng = np.random.default_rng([seed, zlib.crc32(name.encode())])
    if name.endswith("LayerNorm.weight"):
        return (1.0 + 0.05 * rng.standard_normal(shape)).astype(np.float32)
    if name.endswith("LayerNorm.bias"):
        return (0.05 * rng.standard_normal(shape)).astype(np.float32)
    return (0.02 * rng.standard_normal(shape)).astype(np.float32)


def init_model_(model, seed: int = 0):
    """Overwrite every parameter of an HF module with the deterministic values."""
    import torch
    with torch.no_grad():
        for name, p in model.named_parameters():
            p.copy_(torch.from_numpy(param_value(seed, name, tuple(p.shape))))
    return model


def token_batch(batch: int, length: int, seed: int = 0, min_len: int = 4, vocab: int = 30522, fixed: bool = False):
    """(input_ids, attention_mask) int64 [batch, length] in the collator format."""
    rng = np.random.default_rng(seed)
    ids = np.zeros((batch, length), np.int64)
    mask = np.zeros((batch, length), np.int64)
    for b in range(batch):
        n = length if fixed else int(rng.integers(min_len, length + 1))
        ids[b, 0] = 101
        ids[b, 1:n - 1] = rng.integers(1000, vocab, size=n - 2)
        ids[b, n - 1] = 102
        mask[b, :n] = 1
    return ids, mask
