"""Query tower leg of bench.py alone (bench_legs.run_query_encode): batches 8 / 128 / 512 of 32-token
queries, eager vs hipGraph replay.  DRT_LIB selects an A/B build of libdrt_hip.so."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_legs  # noqa: E402

dev = torch.device("cuda", 0)
print(json.dumps(bench_legs.run_query_encode(dev, batches=(8, 128, 512))), flush=True)
