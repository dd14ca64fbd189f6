#!/usr/bin/env python3
"""Encode-leg A/B (bench_legs.run: bf16 BERT-base passages, batch 512 x 128 tokens, the product's
HipBertEncoder) for one library variant (DRT_LIB=<variants/libdrt_hip.X.so>, tools/build_variant.sh), plus a
checksum of the pooled reps to confirm variants that must agree bit for bit.
usage: DRT_LIB=... python tools/encode_ab.py [steps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_legs  # noqa: E402


def main(steps=10):
    dev = torch.device("cuda", 0)
    r = bench_legs.run(dev, steps=steps)
    print(json.dumps({"lib": os.path.basename(os.environ.get("DRT_LIB", "product")), "passages_s": r["value"],
                      "ms_per_step": r["ms_per_step"], "frac": r["roofline"]["frac"]}), flush=True)


if __name__ == "__main__":
    main(*[int(v) for v in sys.argv[1:]])
