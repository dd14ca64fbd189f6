"""Encode leg A/B (512 x 128): the shipped two half-batch streams at equal priority vs the first half's
stream at high priority (hardware queue priority: the second half's work-groups fill the CUs the first
half leaves idle instead of competing for them).  Outputs checked equal."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(rounds=3, steps=8, B=512):
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd.model.encoder import HipBertEncoder
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(m, dev)
    del m
    L = 128
    ids = torch.randint(1000, 30522, (B, L), device=dev)
    mask = torch.ones((B, L), dtype=torch.int64, device=dev)
    enc(ids, mask)
    base_streams = enc._streams
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    variants = {
        "equal": base_streams,
        "first_high": [torch.cuda.Stream(dev, priority=-1), torch.cuda.Stream(dev, priority=0)],
        "second_high": [torch.cuda.Stream(dev, priority=0), torch.cuda.Stream(dev, priority=-1)],
    }
    ref = None
    res, same = {}, {}
    for _ in range(rounds):
        for name, sts in variants.items():
            enc._streams = sts
            out = enc(ids, mask).clone()
            torch.cuda.synchronize()
            if ref is None:
                ref = out
            same[name] = bool(torch.equal(out, ref))
            t0 = time.perf_counter()
            for _ in range(steps):
                enc.pool(enc(ids, mask), mask, "first")
            torch.cuda.synchronize()
            res.setdefault(name, []).append(round(steps * B / (time.perf_counter() - t0), 1))
    print(json.dumps({"median": {k: sorted(v)[len(v) // 2] for k, v in res.items()}, "rounds": res,
                      "bit_identical": same}))


if __name__ == "__main__":
    main()
