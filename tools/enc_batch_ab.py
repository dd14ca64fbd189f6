"""Encode leg per batch size and stream split (passages/s, bf16 BERT-base, L = 128):
batch 512 / 1024 / 2048, with and without HipBertEncoder's two-stream halves, interleaved rounds."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(rounds=3, steps=6):
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd.model.encoder import HipBertEncoder
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(m, dev)
    L = 128
    res = {}
    cfgs = [(512, True), (512, False), (1024, True), (1024, False), (2048, True)]
    for _ in range(rounds):
        for B, split in cfgs:
            ids = torch.randint(1000, 30522, (B, L), device=dev)
            mask = torch.ones((B, L), dtype=torch.int64, device=dev)
            enc.split_streams = split
            enc.pool(enc(ids, mask), mask, "first")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                enc.pool(enc(ids, mask), mask, "first")
            torch.cuda.synchronize()
            pps = steps * B / (time.perf_counter() - t0)
            res.setdefault(f"b{B}_{'split' if split else 'one'}", []).append(round(pps, 1))
    print(json.dumps({k: sorted(v)[len(v) // 2] for k, v in res.items()} | {"all": res}))


if __name__ == "__main__":
    main()
