"""CPU: the torch restatement of the training-dropout hash (csrc/drt_common.h drop_hash24) used by
tests/test_train_tower_gpu.py as its mask generator, against plain Python uint64 arithmetic."""
import numpy as np

from tests.test_train_tower_gpu import _hash24_py, _keep_torch


def test_dropout_hash_torch_restatement_cpu():
    import torch
    rng = np.random.default_rng(0)
    idx = rng.integers(0, 1 << 40, size=2000)
    for seed, site in ((0, 0), (12345678901234, 7), ((1 << 62) - 1, 49)):
        want = np.array([_hash24_py(seed, site, int(i)) >= int(np.float32(0.1) * np.float32(16777216.0))
                         for i in idx])
        got = _keep_torch(seed, site, torch.from_numpy(idx), 0.1).numpy()
        assert (got == want).all()
