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

Launch: python bench.py [--gpus N --steps K --warmup W].  For N > 1 either
under torch.distributed.run (WORLD_SIZE must then equal N) or directly: with
WORLD_SIZE unset, `python bench.py --gpus N` starts the N ranks itself (one
process per GPU, RCCL over xGMI) through a torch.distributed.run child launched
BEFORE anything touches the GPU, and exits with its status (launch()).
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
    # 32 steps = two full groups of 16 batches on the grouped path (search.GROUP_QUERIES); the warm-up
    # runs one full group too (first-use allocations of the group-sized buffers)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--n-corpus", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--qb", type=int, default=128)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-encode", action="store_true",
                    help="skip the encode leg (passages/sec of the bf16 BERT-base passage tower, every rank)")
    ap.add_argument("--no-evaluate", action="store_true", help="skip the C2 Trainer.evaluate leg")
    ap.add_argument("--c2-passages", type=int, default=1_000_000, help="corpus size of the C2 evaluate leg")
    ap.add_argument("--group-queries", type=int, default=-1,
                    help="queries per group of batches in search_batches (0 = per-batch path; default: "
                         "search.GROUP_QUERIES)")
    ap.add_argument("--protocol", choices=["global_tau", "per_shard"], default="global_tau",
                    help="N > 1 exchange protocol (per_shard = exact top-k per shard + merge)")
    ap.add_argument("--order", choices=["exact", "fp32"], default="exact",
                    help="exact: the canonical exact-score order (search.EXACT_ORDER, the product default); "
                         "fp32: the scan's fp32 order (A/B of the refine stage's cost)")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, join the process group, report n_gpus and exit without touching "
                         "the GPU (tests/test_bench_launch_cpu.py)")
    return ap.parse_args()


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args):
    """Start one rank per GPU when asked for N > 1 GPUs outside a launcher.

    Returns when this process IS a rank (WORLD_SIZE set by torch.distributed.run, the driver's form
    for N > 1) or N = 1; otherwise runs `python -m torch.distributed.run --nproc-per-node N bench.py
    ...` as a child and exits with its status.  This process has not initialised the GPU (no HIP
    call has been made yet), and the ranks are a child process, not an exec."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            sys.stderr.write(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}; launch one rank per GPU\n")
            sys.exit(2)
        return
    if args.gpus <= 1:
        return
    import subprocess
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    rc = subprocess.call(cmd, env=env)
    sys.exit(rc)


def launch_check(args):
    """--launch-check: every rank joins the process group (gloo, no GPU) and rank 0 reports how many
    ranks the launch produced."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    seen = world
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.ones(1)
        dist.all_reduce(t)
        seen = int(t.item())
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_joined": seen,
                          "backend": os.environ.get("DRT_BENCH_BACKEND", "nccl")}), flush=True)


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


CORPUS_BLOCK_ROWS = 1 << 20


def corpus_block_seed(b):
    """Seed of global row block b (rows [b * CORPUS_BLOCK_ROWS, (b + 1) * CORPUS_BLOCK_ROWS))."""
    return (1234 << 32) + b


def gen_shard(n_total, world, rank, d, device):
    """Seeded N(0,1) bf16 corpus rows of this rank's contiguous shard (generated in HBM).  Rows are
    generated by GLOBAL row block ("seed 1234 by row-block counter"), so the union of the
    W shards is the same 10M-row corpus for every W and the 1/2/4/8-GPU lines search the same rows."""
    import torch
    per = -(-n_total // world)
    lo = min(n_total, rank * per)
    hi = min(n_total, lo + per)
    g = torch.Generator(device=device)
    shard = torch.empty((hi - lo, d), dtype=torch.bfloat16, device=device)
    B = CORPUS_BLOCK_ROWS
    for b in range(lo // B, -(-hi // B)):
        a0, b0 = b * B, min(n_total, (b + 1) * B)
        g.manual_seed(corpus_block_seed(b))
        blk = torch.randn((b0 - a0, d), generator=g, device=device, dtype=torch.float32).to(torch.bfloat16)
        x0, x1 = max(lo, a0), min(hi, b0)
        shard[x0 - lo: x1 - lo] = blk[x0 - a0: x1 - a0]
        del blk
    return shard, lo, hi


def _cpu_threads():
    import torch
    info = {"host_cpu_count": os.cpu_count(), "torch_threads": torch.get_num_threads()}
    try:
        from threadpoolctl import threadpool_info
        blas = [i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"]
        info["blas_threads"] = max(blas) if blas else None
    except Exception:
        info["blas_threads"] = None
    return info


def _tie_check(q, shard, gi, ci):
    """Every (query, rank) where the GPU's id differs from the CPU baseline's: recompute both rows'
    scores in fp64 from the same bf16 rows and report the largest gap.  A gap within fp32 summation
    noise (<= 1e-3, north_star's score tolerance) means the two rows are a near-tie that fp32 BLAS
    and the MFMA sum order rank differently -- not a wrong answer."""
    import numpy as np
    qi, ri = np.nonzero(gi != ci)
    if qi.size == 0:
        return 0, 0.0
    import torch
    ids = np.unique(np.concatenate([gi[qi, ri], ci[qi, ri]]))
    ids = ids[ids >= 0]
    rows = shard[torch.from_numpy(ids).to(shard.device)].double().cpu().numpy()
    pos = {int(x): j for j, x in enumerate(ids)}
    qd = q.astype(np.float64)
    gap = 0.0
    for a, b in zip(qi, ri):
        sg = float(qd[a] @ rows[pos[int(gi[a, b])]]) if gi[a, b] >= 0 else -np.inf
        sc = float(qd[a] @ rows[pos[int(ci[a, b])]]) if ci[a, b] >= 0 else -np.inf
        gap = max(gap, abs(sg - sc))
    return int(qi.size), gap


def _quiesce_gc():
    """Collect, then freeze every object alive so far (setup, earlier legs, the CPU baselines'
    imports) into the collector's permanent generation: a full collection over that heap inside a
    timed region is harness cost, not the path's (it was 0.215 s of the recipe leg's three timed
    steps, 165 vs 119 ms per step, profiles/r04ad_*).  Objects the timed code creates are still
    collected as usual."""
    import gc
    gc.collect()
    gc.freeze()


def cpu_baseline(args, shard, queries, gpu_result):
    """The oracle (numpy fp32 BLAS, like faiss IndexFlatIP's sgemm + top-k) timed on the host
    cores against the SAME 10M-row corpus the GPU searched: the shard streams to host in
    262,144-row chunks (bf16 -> fp32 conversion untimed, as building a faiss index would be),
    and ONE query batch is scored and selected chunk by chunk (timed).  Also checks the GPU's
    top-k of that batch against the CPU result at full size: every differing (query, rank) is
    recomputed in fp64 and must be a near-tie (|gap| <= 1e-3)."""
    import numpy as np
    from oracle.search_oracle import ip_topk, merge_topk
    thr = _cpu_threads()
    q = queries.float().cpu().numpy()
    n = shard.shape[0]
    chunk = 262144
    best_s = best_i = None
    t_comp = 0.0
    for a in range(0, n, chunk):
        pc = shard[a: a + chunk].float().cpu().numpy()
        t0 = time.perf_counter()
        cs, ci = ip_topk(q, pc, args.k, id_offset=a, chunk=pc.shape[0], dtype=np.float32)
        if best_s is None:
            best_s, best_i = cs, ci
        else:
            best_s, best_i = merge_topk(np.stack([best_s, cs]), np.stack([best_i, ci]), args.k)
        t_comp += time.perf_counter() - t0
    gs, gi = gpu_result
    gi = gi.cpu().numpy()
    gs = gs.cpu().numpy()
    same = float((gi == best_i).mean())
    n_mis, gap = _tie_check(q, shard, gi, best_i)
    # parity against the fp64 evaluator (exact products; the canonical order's definition), untimed
    b64_s = b64_i = None
    for a in range(0, n, chunk):
        pc = shard[a: a + chunk].double().cpu().numpy()
        cs, ci = ip_topk(q, pc, args.k, id_offset=a, chunk=pc.shape[0], dtype=np.float64, out_dtype=np.float64)
        if b64_s is None:
            b64_s, b64_i = cs, ci
        else:
            b64_s, b64_i = merge_topk(np.stack([b64_s, cs]), np.stack([b64_i, ci]), args.k)
    same64 = float((gi == b64_i).mean())
    cores = int(thr["blas_threads"] or thr["torch_threads"])
    value = q.shape[0] / t_comp
    return {
        "value": round(value, 3),
        "unit": "queries/s",
        "cores": cores,
        "kind": "port",
        "sample": (f"oracle/search_oracle.ip_topk fp32 (numpy BLAS, {cores} threads = the box's CPU share per GPU; "
                   f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS')}) on one batch of "
                   f"{q.shape[0]} queries against the full {n}-row bf16 corpus streamed from the GPU in "
                   f"{chunk}-row chunks (fp32 conversion untimed); {t_comp:.1f} s of compute"),
        # the reference runs faiss with OMP_NUM_THREADS=40 (run.sh:24); linear scaling from the measured
        # threads is an upper bound for that configuration on this host
        "projected_40_threads_upper_bound": round(value * 40 / max(1, cores), 3),
        **thr,
        "parity_vs_gpu": {"ids_equal_frac": round(same, 6),
                          "max_abs_score_diff": float(np.abs(gs - best_s).max()),
                          "n_mismatch": n_mis,
                          "max_tie_gap_fp64": gap,
                          "all_mismatches_near_ties": bool(gap <= 1e-3)},
        # the same batch against the fp64 evaluator (oracle ip_topk in float64 over the full corpus)
        "parity_vs_gpu_fp64": {"ids_equal_frac": round(same64, 6),
                               "n_mismatch": int((gi != b64_i).sum()),
                               "max_abs_score_diff": float(np.abs(gs.astype(np.float64) - b64_s).max()),
                               "scores_equal_fp32_frac": round(float((gs == b64_s.astype(np.float32)).mean()), 6)},
    }


def union_parity(args, queries, gpu_result, device, nq=8):
    """N > 1 (rank 0, untimed, after the timed region): the first `nq` queries of the first timed batch
    against the fp64 oracle over the UNION of the shards -- the n_corpus rows regenerated block by block
    from the same per-block seeds every rank generated its shard from (gen_shard) -- so the sharded
    protocol's merged top-k is checked at full size like the N = 1 line's cpu_baseline parity."""
    import numpy as np
    import torch
    from oracle.search_oracle import ip_topk, merge_topk
    q = queries[:nq].float().cpu().numpy()
    n, d, B, chunk = args.n_corpus, queries.shape[1], CORPUS_BLOCK_ROWS, 262144
    g = torch.Generator(device=device)
    best_s = best_i = None
    t0 = time.perf_counter()
    for b in range(-(-n // B)):
        a0, b0 = b * B, min(n, (b + 1) * B)
        g.manual_seed(corpus_block_seed(b))
        blk = torch.randn((b0 - a0, d), generator=g, device=device, dtype=torch.float32).to(torch.bfloat16)
        for c in range(0, b0 - a0, chunk):
            pc = blk[c: c + chunk].double().cpu().numpy()
            cs, ci = ip_topk(q, pc, args.k, id_offset=a0 + c, chunk=pc.shape[0], dtype=np.float64,
                             out_dtype=np.float64)
            if best_s is None:
                best_s, best_i = cs, ci
            else:
                best_s, best_i = merge_topk(np.stack([best_s, cs]), np.stack([best_i, ci]), args.k)
        del blk
    gs, gi = gpu_result
    gs, gi = gs[:nq].cpu().numpy(), gi[:nq].cpu().numpy()
    return {"queries": nq, "rows": n, "ids_equal_frac": round(float((gi == best_i).mean()), 6),
            "n_mismatch": int((gi != best_i).sum()),
            "max_abs_score_diff": float(np.abs(gs.astype(np.float64) - best_s).max()),
            "check_s": round(time.perf_counter() - t0, 1),
            "what": "merged sharded top-k vs oracle/search_oracle.ip_topk in fp64 over the union of the shards"}


def encode_cpu_baseline(batch=32, L=128, min_seconds=10.0):
    """torch-CPU fp32 DRModel.encode (the reference's arithmetic: HF BertModel fp32 + [CLS]
    pooling through this build's DRModelForInference, which is pinned to the reference's
    golden reps on CPU), BERT-base random init, B = 32, L = 128."""
    import torch
    from transformers import BertConfig, BertModel
    from denseretrievaltoolkits_amd.model.biencoder import DRModelForInference
    thr = _cpu_threads()
    torch.manual_seed(0)
    lm = BertModel(BertConfig(), add_pooling_layer=False).eval()
    m = DRModelForInference(lm_q=lm, lm_p=lm, pooling="first").eval()
    ids = torch.randint(1000, 30522, (batch, L), dtype=torch.int64)
    ids[:, 0], ids[:, -1] = 101, 102
    item = {"input_ids": ids, "attention_mask": torch.ones((batch, L), dtype=torch.int64)}
    with torch.no_grad():
        m(passage=item)
        t0 = time.perf_counter()
        steps = 0
        while time.perf_counter() - t0 < min_seconds:
            m(passage=item)
            steps += 1
    el = time.perf_counter() - t0
    return {"value": round(steps * batch / el, 2), "unit": "passages/s", "cores": int(thr["torch_threads"]),
            "kind": "port", "sample": f"{steps} batches of {batch} x {L} tokens, fp32, {el:.1f} s", **thr}


def pmc_traffic(args, world, shape=None):
    """HBM bytes per launch of the dominant kernel from a committed rocprofv3 PMC pass
    (tools/pmc_traffic.py -> profiles/*_pmc_traffic.json) measured on this exact
    configuration (``shape`` = (queries, rows) of a grouped launch); None when no such measurement
    exists."""
    import glob
    want = {"n_corpus": args.n_corpus, "world": world, "qb": args.qb, "k": args.k, "dim": args.dim}
    if shape is not None:
        want.update(launch_queries=int(shape[0]), launch_rows=int(shape[1]))
    import re

    def order(f):   # newest measurement first: round, then tag (a..z, aa..az, ba.. : by length, then letters)
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")), key=order, reverse=True):
        try:
            with open(f) as fh:
                rec = json.load(fh)
        except (OSError, ValueError):
            continue
        if rec.get("config") == want:
            return int(rec["traffic_bytes_per_launch"]), os.path.basename(f)
    return None, None


def launch_shapes(steps, qb, grouped, group_queries, rows, chunks=None):
    """(queries, rows) of every filter-scan launch in the timed region: one launch per batch over the
    shard on the per-batch path; on the grouped one, per group of batches (search._groups: at most
    group_queries queries) one launch over the shard, or one per row chunk (search.group_chunks; a
    sharded index splits every shard into the same count, ShardedFlatIP.group_chunks)."""
    if not grouped:
        return [(qb, rows)] * steps
    sizes, cur = [], 0
    for _ in range(steps):
        if cur and cur + qb > group_queries:
            sizes.append(cur)
            cur = 0
        cur += qb
    if cur:
        sizes.append(cur)
    parts = [b - a for a, b in chunks] if chunks else [rows]
    return [(q, r) for q in sizes for r in parts]


def scan_roofline(d, k, kc, shapes, grouped, launch_ms_total):
    """Roofline of the filter-scan launches of the timed region from their own shapes:
    per launch over N_s rows with Q queries, bytes = N_s d 2 + Q d 2 + the result lists (Q k 12 per
    batch; the grouped launch writes packed [Q, kc + 1] u64 lists), flops = 2 Q N_s d; t_roof =
    max(bytes / 8 TB/s, flops / 2.5 PF/s) summed over the launches; frac = t_roof / measured;
    achieved = the bound's quantity / measured.  A grouped launch (Q = 2048) is MFMA-side, a
    128-query pass HBM-bound."""
    byts = sum(r * d * 2 + q * d * 2 + (q * (kc + 1) * 8 if grouped else q * k * 12) for q, r in shapes)
    flops = sum(2 * q * r * d for q, r in shapes)
    t_hbm = byts / (HBM_PEAK_GBS * 1e9)
    t_mfma = flops / (BF16_PEAK_TFLOPS * 1e12)
    t = launch_ms_total * 1e-3
    hbm = t_hbm >= t_mfma
    n = max(1, len(shapes))
    return {
        "bound": "hbm" if hbm else "mfma",
        "achieved": round(byts / t / 1e9 if hbm else flops / t / 1e12, 1),
        "peak": HBM_PEAK_GBS if hbm else BF16_PEAK_TFLOPS,
        "unit": "GB/s" if hbm else "TFLOP/s",
        "frac": round(max(t_hbm, t_mfma) / t, 4),
        "launches": len(shapes),
        "launch_shapes": sorted(set(shapes)),
        "avg_launch_ms": round(launch_ms_total / n, 4),
        "alg_bytes_per_launch": int(byts // n),
        "alg_flops_per_launch": int(flops // n),
    }


def per_shape(d, k, kc, shapes, grouped, each_ms):
    """Average launch time and roofline fraction of every launch shape of the timed region (its
    launches matched to the shapes in issue order; None when the counts differ, e.g. a redone batch)."""
    if each_ms is None or len(each_ms) != len(shapes):
        return None
    acc = {}
    for sh, ms in zip(shapes, each_ms):
        acc.setdefault(tuple(sh), []).append(ms)
    out = []
    for (q, r), v in sorted(acc.items(), reverse=True):
        rf = scan_roofline(d, k, kc, [(q, r)] * len(v), grouped, sum(v))
        out.append({"queries": q, "rows": r, "launches": len(v), "avg_launch_ms": round(sum(v) / len(v), 4),
                    "bound": rf["bound"], "frac": rf["frac"], "achieved": rf["achieved"], "unit": rf["unit"]})
    return out


def search_record(args, world, grouped, group_queries, kc, elapsed_s, launch_ms_total, launches, traffic,
                  chunks=None, each_ms=None):
    """The headline JSON record of the search leg (rank 0).  ``chunks``: the row ranges of rank 0's
    group filter launches (search.group_chunks / ShardedFlatIP.group_chunks; rank 0 holds the largest
    shard)."""
    d, k, qb = args.dim, args.k, args.qb
    per = -(-args.n_corpus // world)
    shapes = launch_shapes(args.steps, qb, grouped, group_queries, per, chunks)
    rf = scan_roofline(d, k, kc, shapes, grouped, launch_ms_total)
    # launches of more than 128 queries run the 32-queries-per-wave kernel (search.hip, launch_scan_d)
    kname = "ip_scan32r_kernel" if grouped and group_queries > 128 and d <= 768 else "ip_scan16r_kernel"
    rf = {"kernel": "%s<%d> (csrc/search.hip)" % (kname, d), **rf}
    if launches != len(shapes):
        rf["launches_counted"] = launches   # the profiler's count (differs only if a batch was redone)
    ps = per_shape(d, k, kc, shapes, grouped, each_ms)
    if ps is not None and len(ps) > 1:
        for e in ps:   # PMC traffic of each shape where a record of that launch shape exists
            e["traffic"], e["traffic_source"] = pmc_traffic(args, world, (e["queries"], e["rows"]) if grouped else None)
        rf["per_shape"] = ps   # rank 0's launches by shape (the line's avg_launch_ms mixes them)
    # PMC traffic (tools/pmc_traffic.py) of this configuration's dominant launch shape
    tb, tsrc = traffic
    rf["traffic"] = tb
    rf["traffic_source"] = tsrc
    if world == 1:
        path = ("FlatIPIndex.search_batches (certified, pipelined; " +
                (f"grouped: one sample launch, the filter over all {group_queries} queries of a group (16 query "
                 f"blocks sharing each corpus tile through L2) as {len(chunks or [0])} launch(es) over row chunks "
                 "of <= search.GROUP_CHUNK_ROWS rows, one merge of the chunks' lists per group)" if grouped else
                 "per batch: sample scan + k-th selection, one filter launch, select, canonical-order stage)"))
    else:
        path = (f"ShardedFlatIP.search_batches ({args.protocol}, certified, pipelined; " +
                (f"grouped: one sample launch, sample-list all-gather, the filter over all {group_queries} "
                 f"queries of a group as {len(chunks or [0])} launch(es) over row chunks of the shard, packed "
                 "all-gather of every chunk's lists and one merge per group)" if grouped else
                 "per batch: per-shard exact top-k, all-gather, merge)"))
    qps = args.steps * qb / elapsed_s
    return {
        "metric": "queries/sec@top-1000, 10Mx768 corpus (BASELINE: passages encoded/sec + queries/sec@top-1000, "
                  "10Mx768 corpus, 1/2/4/8 GPU)",
        "value": round(qps, 2),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_s / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic: N(0,1) corpus and queries rounded to bf16, generated in HBM (seeded per global "
                "1M-row block: the same corpus at every GPU count)",
        "config": {
            "workload": f"exact IP top-{k}, {args.n_corpus} x {d} bf16 corpus row-sharded over {world} GPU(s), "
                        f"loader batch {qb} queries" + (f", searched in groups of {group_queries}" if grouped else
                                                        ", searched per batch"),
            "n_corpus": args.n_corpus, "dim": d, "query_batch": qb, "k": k,
            "queries_per_filter_launch": group_queries if grouped else qb,
            "parallelism": f"row-shard x{world}",
            "path": path,
        },
        "roofline": rf,
    }


def encode_leg(args, device):
    import bench_legs
    return bench_legs.run(device)


def main():
    args = parse()
    launch(args)
    if args.launch_check:
        launch_check(args)
        return
    import torch
    import torch.distributed as dist
    rank, world, local = init_dist(args.gpus)
    dev = torch.device("cuda", local)
    from denseretrievaltoolkits_amd import _native, kernels

    lib = _native.load()
    d, k, qb = args.dim, args.k, args.qb
    # host-only setup first (imports, the collector's pass over the import heap), so the GPU work that follows
    # -- corpus generation, row statistics, the warm-up -- runs back to back (the 17-29 ms host pauses between
    # them are gone from the trace; the first timed launches still run 3.3 -> 3.0 ms, profiles/r06ramp/)
    from denseretrievaltoolkits_amd import search as srch
    from denseretrievaltoolkits_amd.search import FlatIPIndex, ShardedFlatIP
    _quiesce_gc()
    shard, lo, hi = gen_shard(args.n_corpus, world, rank, d, dev)
    n_local = hi - lo
    nsteps = args.warmup + args.steps
    gq = torch.Generator(device=dev)
    gq.manual_seed(5678)
    queries = torch.randn((nsteps, qb, d), generator=gq, device=dev).to(torch.bfloat16)

    gloo = world > 1 and dist.get_backend() == "gloo"
    srch.EXACT_ORDER = args.order == "exact"
    if args.group_queries == 0:
        srch.GROUP_MIN_ROWS = 1 << 62          # one-GPU: per-batch path
        srch.GROUP_QUERIES = qb                 # several GPUs: one batch per group
    elif args.group_queries > 0:
        srch.GROUP_QUERIES = args.group_queries
        srch.GROUP_MIN_ROWS = 0                 # one-GPU: grouped path too, at any shard size
    # the product path: the same index objects and certified, pipelined batch search that
    # BaseFaissIPRetriever.batch_search / Trainer.evaluate use (search.py); every query
    # certified exact inside the timed region (an uncertified one is rescanned there)
    if world == 1:
        index = FlatIPIndex.from_rows(shard)

        def run(first, last):
            return index.search_batches([queries[j] for j in range(first, last)], k)
    else:
        index = ShardedFlatIP(d, device=dev, protocol=args.protocol)
        index.local = FlatIPIndex.from_rows(shard)
        index.sync_offsets()
        assert index.offset == lo and index.ntotal == args.n_corpus

        def run(first, last):
            return index.search_batches([queries[j] for j in range(first, last)], k)

    # the collector is quiesced BEFORE the warm-up, so the timed steps follow the warm-up's last launch
    # with no host pause: a 49 ms collection between them left the GPU idle long enough that the first
    # timed launches ran 10-20 % slow (clocks ramping back: 3.45, 3.53, 3.24 ms vs 2.85-2.98 back to back,
    # profiles/r05ap/kernel_stats)
    _quiesce_gc()
    run(0, args.warmup)
    torch.cuda.synchronize()
    local_index = index if world == 1 else index.local

    def fallbacks():
        return index.group_fallbacks if world == 1 else index.fallbacks

    def timed(first, last):
        """Batches [first, last) between barriers + syncs: (results, max-over-ranks elapsed s, filter-launch
        ms summed over the launches (slowest rank's average x count), launches, counter deltas)."""
        res0, fb0, unc0 = local_index.resolved, fallbacks(), index.order_uncertified
        lib.drt_profile_enable(_native.PROF_SCAN, 1)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = run(first, last)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        lib.drt_profile_enable(_native.PROF_SCAN, 0)
        cap = 1 << 14
        each = (_native.ctypes.c_double * cap)()
        cnt = _native.c_i64(0)
        _native.check(lib.drt_profile_read_each(_native.PROF_SCAN, each, cap, _native.ctypes.byref(cnt)),
                      "drt_profile_read_each")
        each_ms = [float(each[j]) for j in range(min(cap, int(cnt.value)))]
        elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
        scan_ms = torch.tensor([sum(each_ms) / max(1, cnt.value)], dtype=torch.float64, device=dev)
        if world > 1:
            if gloo:
                elapsed, scan_ms = elapsed.cpu(), scan_ms.cpu()
            dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
            dist.all_reduce(scan_ms, op=dist.ReduceOp.MAX)
        counters = (local_index.resolved - res0, fallbacks() - fb0, index.order_uncertified - unc0)
        timed.each_ms = each_ms   # this rank's launches, in issue order (per-shape averages in the record)
        return res, float(elapsed.item()), float(scan_ms.item()) * int(cnt.value), int(cnt.value), counters

    results, el, scan_ms_total, launches, (n_resolved, n_fallback, n_unc) = timed(args.warmup, nsteps)
    each_ms = timed.each_ms
    grouped = index._use_groups()
    sub = None
    if world > 1 and grouped:
        # SURVEY §8(d)'s HBM-bound configuration beside the product default: the same protocol with one
        # 128-query batch per group (one filter launch per batch)
        gq_saved = srch.GROUP_QUERIES
        srch.GROUP_QUERIES = qb
        _quiesce_gc()
        run(0, 1)
        _, el1, ms1, n1, _ = timed(args.warmup, nsteps)
        srch.GROUP_QUERIES = gq_saved
        if rank == 0:
            sub = search_record(args, world, True, qb, kernels.refine_width(k), el1, ms1, n1, (None, None),
                                chunks=index.group_chunks())
            sub = {"value": sub["value"], "ms_per_step": sub["ms_per_step"],
                   "config": "one 128-query batch per group (per-batch global-threshold protocol)",
                   "roofline": sub["roofline"]}

    out = None
    if rank == 0:
        chunks = srch.group_chunks(n_local) if world == 1 else index.group_chunks()
        shape = (srch.GROUP_QUERIES, max(b - a for a, b in chunks)) if grouped else None
        out = search_record(args, world, grouped, srch.GROUP_QUERIES, kernels.refine_width(k), el,
                            scan_ms_total, launches, pmc_traffic(args, world, shape), chunks=chunks,
                            each_ms=each_ms)
        if sub is not None:
            out["per_batch_qb%d" % qb] = sub
        out["order"] = ("canonical: exact-score re-rank of each query's near-tie window (fp64 sums of the bf16 "
                        "products, ties by id), the product default" if args.order == "exact" else
                        "fp32 scan order (A/B leg)")
        out["order_uncertified_queries"] = int(n_unc)
        out["uncertified_queries_resolved"] = int(n_resolved)
        out["global_tau_fallback_batches"] = int(n_fallback)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, shard, queries[args.warmup], results[0])
        elif world > 1 and not args.no_cpu_baseline:
            out["parity_union_fp64"] = union_parity(args, queries[args.warmup], results[0], dev)
    # the search leg's 15 GB corpus, index and results leave HBM before the model legs (the training
    # legs' torch baselines reserve ~140 GB)
    del shard, queries, results, index, local_index
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
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
        import bench_legs as bench_encode
        if not args.no_cpu_baseline:
            out["encode"]["cpu_baseline"] = encode_cpu_baseline()
        def leg(fn, *a, **kw):   # each leg starts from an empty cache and a frozen heap
            _quiesce_gc()
            r = fn(*a, **kw)
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            return r
        out["rerank"] = leg(bench_encode.run_rerank, dev)
        out["query_encode"] = leg(bench_encode.run_query_encode, dev)
        out["train_scores"] = leg(bench_encode.run_train_scores, dev)
        out["train_step"] = leg(bench_encode.run_train_step, dev)
        # the reference recipe's shapes (run.sh:16-19: train_n_passages 8, p_max_len 156) at batch 128
        out["train_step_recipe"] = leg(bench_encode.run_train_step, dev, bq=128, n=8, p_len=156)
        if not args.no_evaluate:
            out["evaluate_c2"] = leg(bench_encode.run_evaluate_c2, dev, n_passages=args.c2_passages)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
