#!/usr/bin/env python3
"""Headline benchmark: queries/sec @ top-1000 over a 10M x 768 bf16 corpus.

BASELINE.json metric: "passages encoded/sec + queries/sec@top-1000, 10M x 768
corpus, 1/2/4/8 GPU".  `value` is the search half (queries/sec@top-1000, the
north-star path: brute-force Q.D^T + top-k, BaseFaissIPRetriever.search,
DRT/evaluator/index.py:31-33); the encode half is reported beside it under
"encode" (passages/sec of the bf16 BERT-base passage
tower, DRModel.encode, DRT/model/biencoder.py:127-151), timed on every rank
after the search leg (weak scaling: each rank encodes its own batches).

One step = one query batch (Qb = 128, the reference's eval batch,
arguments.py:189) searched exactly against the WHOLE corpus (k = 1000):
every rank scans its contiguous row shard (10M / N rows, resident in HBM).
For N > 1 the shards run the global-threshold protocol (search.py
ShardedFlatIP): all-gather of the tiny per-shard sample lists -> one corpus
threshold, filter scan of the shard against it, all-gather of the packed
per-shard top-k (u64 score-key|id) and a device merge that certifies
exactness; an uncertified batch is redone with the per-shard exact path
inside the timed region.  The corpus is fixed as N grows ("scaling": "strong").

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, RCCL).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec, MI355X_MICROARCH.md
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-corpus", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--qb", type=int, default=128)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=1_000_000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-encode", action="store_true",
                    help="skip the encode leg (passages/sec of the bf16 BERT-base passage tower, every rank)")
    ap.add_argument("--scan-variant", type=int, default=0, help="benchmark-only ablation of the scan kernel")
    ap.add_argument("--streams", type=int, default=1,
                    help="HIP streams the query batches rotate over (overlaps one batch's exchange and small "
                         "kernels with the next batch's scan)")
    ap.add_argument("--protocol", choices=["global_tau", "per_shard"], default="global_tau",
                    help="N > 1 exchange protocol (per_shard = exact top-k per shard + merge)")
    return ap.parse_args()


def init_dist(n_gpus):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DRT_BENCH_BACKEND=gloo: rehearsal of the N > 1 logic with several ranks
    # sharing one GPU (collectives staged through host memory; not a measurement)
    backend = os.environ.get("DRT_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return rank, world, local


def gen_shard(n_total, world, rank, d, device):
    """Seeded N(0,1) bf16 corpus rows of this rank's contiguous shard (generated in HBM)."""
    import torch
    per = -(-n_total // world)
    lo = min(n_total, rank * per)
    hi = min(n_total, lo + per)
    g = torch.Generator(device=device)
    g.manual_seed(1234 + rank)
    shard = torch.empty((hi - lo, d), dtype=torch.bfloat16, device=device)
    step = 1 << 20
    for a in range(0, hi - lo, step):
        b = min(hi - lo, a + step)
        shard[a:b] = torch.randn((b - a, d), generator=g, device=device, dtype=torch.float32).to(torch.bfloat16)
    return shard, lo, hi


def cpu_baseline(args):
    """Oracle (numpy, fp32 like faiss IndexFlatIP) on a bounded sample of the same workload."""
    import numpy as np
    from oracle.search_oracle import bf16_round, ip_topk
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:
        cores = os.cpu_count() or 1
    rng = np.random.default_rng(99)
    rows = args.cpu_rows
    p = bf16_round(rng.standard_normal((rows, args.dim), dtype=np.float32))
    q = bf16_round(rng.standard_normal((args.qb, args.dim), dtype=np.float32))
    nb = 0
    t0 = time.perf_counter()
    while True:
        ip_topk(q, p, args.k, chunk=rows, dtype=np.float32)
        nb += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or nb >= 50:
            break
    qps_sample = nb * args.qb / el
    scale = rows / args.n_corpus
    return {
        "value": round(qps_sample * scale, 3),
        "unit": "queries/s",
        "cores": int(cores),
        "kind": "port",
        "sample": (f"oracle/search_oracle.ip_topk fp32 (numpy BLAS) on {nb} batches x {args.qb} queries "
                   f"against a {rows}-row slice ({qps_sample:.1f} q/s), scaled by {rows}/{args.n_corpus} "
                   f"to the full corpus; {el:.1f} s"),
    }


def pmc_traffic(args, world):
    """HBM bytes per launch of the dominant kernel from a committed rocprofv3 PMC pass
    (tools/pmc_traffic.py -> profiles/*_pmc_traffic.json) measured on this exact
    configuration; None when no such measurement exists."""
    import glob
    want = {"n_corpus": args.n_corpus, "world": world, "qb": args.qb, "k": args.k, "dim": args.dim}
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")), reverse=True):
        try:
            with open(f) as fh:
                rec = json.load(fh)
        except (OSError, ValueError):
            continue
        if rec.get("config") == want:
            return int(rec["traffic_bytes_per_launch"]), os.path.basename(f)
    return None, None


def encode_leg(args, device):
    try:
        from denseretrievaltoolkits_amd import bench_encode
    except ImportError:
        return None
    return bench_encode.run(device)


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    rank, world, local = init_dist(args.gpus)
    dev = torch.device("cuda", local)
    from denseretrievaltoolkits_amd import _native, kernels

    lib = _native.load()
    _native.check(lib.drt_scan_variant(args.scan_variant), "drt_scan_variant")
    d, k, qb = args.dim, args.k, args.qb
    shard, lo, hi = gen_shard(args.n_corpus, world, rank, d, dev)
    n_local = hi - lo
    nsteps = args.warmup + args.steps
    gq = torch.Generator(device=dev)
    gq.manual_seed(5678)
    queries = torch.randn((nsteps, qb, d), generator=gq, device=dev).to(torch.bfloat16)

    s_loc = torch.empty((nsteps, qb, k), dtype=torch.float32, device=dev)
    i_loc = torch.empty((nsteps, qb, k), dtype=torch.int64, device=dev)
    st = torch.zeros((nsteps, qb), dtype=torch.int32, device=dev)
    gloo = world > 1 and dist.get_backend() == "gloo"

    def all_gather(t):
        """[world * rows, ...] concatenated all-gather (RCCL on device; host-staged under gloo)."""
        src = t.contiguous().cpu() if gloo else t.contiguous()
        out = torch.empty((world * src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        dist.all_gather_into_tensor(out, src)
        return out.to(dev).view((world,) + tuple(t.shape))

    def step_per_shard(j):
        kernels.ip_topk(queries[j], shard, k, id_offset=lo, resolve=False,
                        out=(s_loc[j], i_loc[j]), status=st[j])
        if world > 1:
            return kernels.topk_merge(all_gather(s_loc[j]), all_gather(i_loc[j]), k)
        return s_loc[j], i_loc[j]

    def step_global_tau(j):
        best = kernels.dist_sample(queries[j], shard, args.n_corpus, k)
        tau = kernels.dist_tau(all_gather(best), k)
        packed = kernels.dist_filter(queries[j], shard, args.n_corpus, k, lo, tau)
        s, i, stj = kernels.merge_packed(all_gather(packed), k, args.n_corpus)
        st[j] = stj
        return s, i

    use_global = world > 1 and args.protocol == "global_tau"
    step = step_global_tau if use_global else step_per_shard

    def fix_failures(first, last):
        """Exact redo of any uncertified query batch (counted inside the timed region).
        Global-tau statuses come from the merged lists, identical on every rank."""
        bad = (st[first:last] != 0).any(dim=1).to(torch.int32)
        if world > 1 and not use_global:
            bad_c = bad.cpu() if gloo else bad
            dist.all_reduce(bad_c, op=dist.ReduceOp.MAX)
            bad = bad_c.to(dev)
        nb = 0
        for j in (torch.nonzero(bad).flatten() + first).tolist():
            if use_global:
                kernels.ip_topk(queries[j], shard, k, id_offset=lo, resolve=True, out=(s_loc[j], i_loc[j]))
                kernels.topk_merge(all_gather(s_loc[j]), all_gather(i_loc[j]), k)
                nb += qb
                continue
            nb += kernels.resolve_failed(queries[j], shard, k, lo, s_loc[j], i_loc[j], st[j])
            if world > 1:
                kernels.topk_merge(all_gather(s_loc[j]), all_gather(i_loc[j]), k)
        return nb

    main_stream = torch.cuda.current_stream(dev)
    streams = [main_stream] + [torch.cuda.Stream(device=dev) for _ in range(max(1, args.streams) - 1)]

    def run_steps(first, last):
        for s in streams[1:]:
            s.wait_stream(main_stream)
        for j in range(first, last):
            with torch.cuda.stream(streams[j % len(streams)]):
                step(j)
        for s in streams[1:]:
            main_stream.wait_stream(s)

    run_steps(0, args.warmup)
    fix_failures(0, args.warmup)
    torch.cuda.synchronize()

    lib.drt_profile_enable(_native.PROF_SCAN, 1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(args.warmup, nsteps)
    n_resolved = fix_failures(args.warmup, nsteps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    lib.drt_profile_enable(_native.PROF_SCAN, 0)
    tot_ms = _native.ctypes.c_double(0.0)
    cnt = _native.c_i64(0)
    _native.check(lib.drt_profile_read(_native.PROF_SCAN, _native.ctypes.byref(tot_ms), _native.ctypes.byref(cnt)),
                  "drt_profile_read")

    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    scan_ms = torch.tensor([tot_ms.value / max(1, cnt.value)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(scan_ms, op=dist.ReduceOp.MAX)
    el = float(elapsed.item())
    scan_ms_v = float(scan_ms.item())

    out = None
    if rank == 0:
        qps = args.steps * qb / el
        # algorithmic bytes of ONE filter-scan launch on the largest shard:
        # corpus shard (per-row d*2 B) + query block + result lists
        per = -(-args.n_corpus // world)
        alg_bytes = per * d * 2 + qb * d * 2 + (qb * (k + 1) * 8 if use_global else qb * k * 12)
        achieved = alg_bytes / (scan_ms_v * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(args, world)
        out = {
            "metric": "queries/sec@top-1000, 10Mx768 corpus (BASELINE: passages encoded/sec + queries/sec@top-1000, 10Mx768 corpus, 1/2/4/8 GPU)",
            "value": round(qps, 2),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic: N(0,1) corpus and queries rounded to bf16, generated in HBM (seeded)",
            "config": {
                "workload": f"exact IP top-{k}, {args.n_corpus} x {d} bf16 corpus row-sharded over {world} GPU(s), "
                            f"query batch {qb}" + (", global-threshold protocol (RCCL all-gather of sample lists "
                                                   "and packed per-shard top-k, device merge)" if use_global else
                                                   (", RCCL all-gather of per-shard top-k + device merge"
                                                    if world > 1 else "")),
                "n_corpus": args.n_corpus, "dim": d, "query_batch": qb, "k": k,
                "parallelism": f"row-shard x{world}",
                "streams": len(streams),
            },
            "roofline": {
                "kernel": "ip_scan16_kernel<768,FILTER,0,8> (csrc/search.hip)",
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "avg_launch_ms": round(scan_ms_v, 4),
                "launches": int(cnt.value),
                "alg_bytes_per_launch": alg_bytes,
            },
            "uncertified_queries_resolved": int(n_resolved),
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args)
    enc = None if args.no_encode else encode_leg(args, dev)
    if enc is not None:
        if world > 1:
            # aggregate over ranks: every rank encodes its own batches; slowest rank sets the rate
            pps = torch.tensor([enc["value"]], dtype=torch.float64, device="cpu" if gloo else dev)
            dist.all_reduce(pps, op=dist.ReduceOp.MIN)
            enc["per_gpu_min"] = float(pps.item())
            enc["value"] = round(float(pps.item()) * world, 1)
            enc["scaling"] = "weak"
            rf = enc["roofline"]
            rf["achieved"] = round(rf["flop_per_passage"] * enc["per_gpu_min"] / 1e12, 1)
            rf["frac"] = round(rf["achieved"] / rf["peak"], 4)
        if out is not None:
            out["encode"] = enc
    if rank == 0 and not args.no_encode and world == 1:
        from denseretrievaltoolkits_amd import bench_encode
        out["rerank"] = bench_encode.run_rerank(dev)
        out["query_encode"] = bench_encode.run_query_encode(dev)
        out["train_scores"] = bench_encode.run_train_scores(dev)
        out["train_step"] = bench_encode.run_train_step(dev)
        # the reference recipe's shapes (run.sh:16-19: train_n_passages 8, p_max_len 156) at batch 128
        out["train_step_recipe"] = bench_encode.run_train_step(dev, bq=128, n=8, p_len=156)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
