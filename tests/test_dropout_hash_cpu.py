"""CPU: the torch restatements of the training-dropout hashes (csrc/drt_common.h drop_hash24 for the
hidden / embedding sites, attn_row_key + attn_mix for the attention probabilities) used by
tests/test_train_tower_gpu.py as mask generators, against plain Python integer arithmetic."""
import numpy as np

from tests.test_train_tower_gpu import _attn_keep_py, _attn_keep_torch, _hash24_py, _keep_torch


def test_dropout_hash_torch_restatement_cpu():
    import torch
    rng = np.random.default_rng(0)
    idx = rng.integers(0, 1 << 40, size=2000)
    for seed, site in ((0, 0), (12345678901234, 7), ((1 << 62) - 1, 49)):
        want = np.array([_hash24_py(seed, site, int(i)) >= int(np.float32(0.1) * np.float32(16777216.0))
                         for i in idx])
        got = _keep_torch(seed, site, torch.from_numpy(idx), 0.1).numpy()
        assert (got == want).all()


def test_attention_dropout_hash_torch_restatement_cpu():
    B, heads, L = 2, 3, 37
    for seed, site, p in ((0, 1, 0.1), (12345678901234, 7, 0.25), ((1 << 62) - 1, 49, 0.1)):
        got = _attn_keep_torch(seed, site, B, heads, L, p, "cpu").numpy()
        for row in range(B * heads * L):
            want = [_attn_keep_py(seed, site, row, key, p) for key in range(L)]
            assert (got.reshape(-1, L)[row] == np.array(want)).all(), row
    # keep rate of the 16-bit threshold and independence of the two halves of a hash
    keep = _attn_keep_torch(5, 3, 8, 12, 128, 0.1, "cpu").numpy()
    assert abs(keep.mean() - 0.9) < 0.002
    even, odd = keep[..., 0::2].ravel(), keep[..., 1::2].ravel()
    assert abs((even & odd).mean() - even.mean() * odd.mean()) < 0.002
