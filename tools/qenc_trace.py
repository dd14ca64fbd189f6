#!/usr/bin/env python3
"""Query tower at one small batch, eager launches, for a rocprofv3 kernel trace (per-kernel
durations and the gaps between them).  usage: python tools/qenc_trace.py [batch] [L] [steps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd.model.encoder import HipBertEncoder
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(m, dev)
    enc.graphs = False
    ids = torch.randint(1000, 30522, (batch, L), device=dev, dtype=torch.int64)
    mask = torch.ones((batch, L), dtype=torch.int64, device=dev)
    for _ in range(3):
        enc.pool(enc(ids, mask), mask, "first")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        enc.pool(enc(ids, mask), mask, "first")
    torch.cuda.synchronize()
    print(f"batch {batch} x {L}: {(time.perf_counter() - t0) / steps * 1e3:.4f} ms per forward", flush=True)


if __name__ == "__main__":
    main()
