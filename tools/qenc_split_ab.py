"""Query tower: two halves on two HIP streams (HipBertEncoder.split_streams) from small token
counts vs one stream, batches 128 / 256 / 512 x 32 tokens, interleaved."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(steps=50):
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd.model.encoder import HipBertEncoder
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    enc = HipBertEncoder.from_hf(m, dev)
    del m
    res = {}
    for batch in (128, 256, 512):
        ids = torch.randint(1000, 30522, (batch, 32), device=dev, dtype=torch.int64)
        mask = torch.ones((batch, 32), dtype=torch.int64, device=dev)
        for rep in range(2):
            for name, smt in (("one_stream", 1 << 40), ("halves", 1024)):
                enc.split_min_tokens = smt
                for _ in range(3):
                    enc.pool(enc(ids, mask), mask, "first")
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    enc.pool(enc(ids, mask), mask, "first")
                torch.cuda.synchronize()
                res.setdefault(f"b{batch}_{name}_ms", []).append(round((time.perf_counter() - t0) / steps * 1e3, 4))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
