"""Encode leg A/B: one 512 x 128 batch per step vs two 256-passage halves on two HIP streams
(independent kernels of the halves can fill each other's per-layer bubbles)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd.model.encoder import HipBertEncoder
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(m, dev)
    B, L = 512, 128
    ids = torch.randint(1000, 30522, (B, L), device=dev)
    mask = torch.ones((B, L), dtype=torch.int64, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    res = {}

    def one():
        enc.pool(enc(ids, mask), mask, "first")

    def halves(parts):
        cur = torch.cuda.current_stream(dev)
        n = B // parts
        for i in range(parts):
            st = streams[i % 2]
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                sl = slice(i * n, (i + 1) * n)
                enc.pool(enc(ids[sl], mask[sl]), mask[sl], "first")
        for st in streams:
            cur.wait_stream(st)

    for name, fn in (("one_512", one), ("two_256_2streams", lambda: halves(2)),
                     ("four_128_2streams", lambda: halves(4)), ("one_512_again", one)):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        res[name] = round(10 * B / (time.perf_counter() - t0), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
