import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import json, torch
from denseretrievaltoolkits_amd import bench_encode, _native
lib = _native.load()
out = {}
for t in (512, 256, 128, 64):
    lib.drt_gemm_large_min_tiles(t)
    r = bench_encode.run_query_encode(torch.device("cuda", 0), batches=(128, 512))
    out[t] = {k: v["eager_ms_per_batch"] for k, v in r.items() if k.startswith("b")}
print(json.dumps(out))
