"""Query-tower forward time (32 tokens, eager) per mid-size GEMM plan (drt_gemm_mid_config):
off (128^2 kernel below the 256^2 threshold) vs the whole-line 256^2 kernel with K split over
~one block per CU, per fp32-partials cap and minimum K-tiles per split; outputs vs the off plan."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from denseretrievaltoolkits_amd import _native, bench_encode  # noqa: E402

CONFIGS = {"off": (1 << 30, 64 << 20, 4), "m256_c64_k4": (256, 64 << 20, 4), "m1k_c64_k4": (1024, 64 << 20, 4),
           "m1k_c32_k4": (1024, 32 << 20, 4), "m1k_c128_k2": (1024, 128 << 20, 2), "m1k_c1_unsplit": (1024, 1, 4)}


def main():
    lib = _native.load()
    dev = torch.device("cuda", 0)
    out = {}
    for name, cfg in CONFIGS.items():
        lib.drt_gemm_mid_config(*cfg)
        r = bench_encode.run_query_encode(dev, batches=(8, 128, 512), steps=30)
        out[name] = {k: v["eager_ms_per_batch"] for k, v in r.items() if k.startswith("b")}
        print(name, out[name], flush=True)
    lib.drt_gemm_mid_config(*CONFIGS["off"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
