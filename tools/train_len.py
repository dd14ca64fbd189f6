"""Training step (C3 leg of bench.py) at the bench shape and at the reference recipe's shapes
(run.sh:16-19: n = 8, p_max_len 156), HIP tower vs HF fp32 autograd."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_legs as bench_encode  # noqa: E402

dev = torch.device("cuda", 0)
print(json.dumps(bench_encode.run_train_step(dev)), flush=True)
print(json.dumps(bench_encode.run_train_step(dev, bq=128, n=8, p_len=156)), flush=True)
