#!/usr/bin/env python3
"""A/B of bench legs for one library variant (DRT_LIB=<variants/libdrt_hip.X.so>, tools/build_variant.sh):
encode (passages/s), train_step (ms), rerank (queries/s), query_encode (queries/s at batch 128).
usage: DRT_LIB=... python tools/legs_ab.py encode train_step rerank query_encode"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_legs  # noqa: E402


def main(legs):
    dev = torch.device("cuda", 0)
    out = {"lib": os.path.basename(os.environ.get("DRT_LIB", "product"))}
    for leg in legs:
        if leg == "encode":
            out[leg] = bench_legs.run(dev)["value"]
        elif leg == "train_step":
            out[leg] = bench_legs.run_train_step(dev)["hip_ms"]
        elif leg == "rerank":
            out[leg] = bench_legs.run_rerank(dev)["value"]
        elif leg == "query_encode":
            out[leg] = bench_legs.run_query_encode(dev)["value"]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
