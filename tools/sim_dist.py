#!/usr/bin/env python3
"""Per-rank compute of the N-GPU search step, simulated on ONE GPU.

Builds the same 10M x 768 corpus as `bench.py --gpus W` (per-rank seeded
shards), precomputes the other ranks' exchanged data once, then times rank
R's own work for each protocol:
  global_tau : dist_sample(own) + dist_tau(all lists) + dist_filter(own) + merge_packed(all parts)
  per_shard  : ip_topk(own shard) + topk_merge(all parts)
Collectives are excluded (they move 13 KB + 1 MB per step); prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--n-corpus", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--qb", type=int, default=128)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--check", action="store_true", help="verify global_tau == per_shard results")
    ap.add_argument("--graph", action="store_true", help="also time the step replayed from a hipGraph")
    ap.add_argument("--group", type=int, default=16, help="batches per group (grouped protocol)")
    a = ap.parse_args()
    import torch
    import bench
    from denseretrievaltoolkits_amd import _native, kernels
    lib = _native.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    W, R, k, qb, N = a.world, a.rank, a.k, a.qb, a.n_corpus
    shards = [bench.gen_shard(N, W, r, a.dim, dev) for r in range(W)]
    g = torch.Generator(device=dev)
    g.manual_seed(5678)
    queries = torch.randn((a.steps, qb, a.dim), generator=g, device=dev).to(torch.bfloat16)
    out = {"world": W, "rank": R, "n_corpus": N, "qb": qb, "k": k, "steps": a.steps}

    # other ranks' exchanged data, per step
    lists = [torch.stack([kernels.dist_sample(queries[j], sh, N, k) for sh, _, _ in shards]) for j in range(a.steps)]
    taus = [kernels.dist_tau(l, k) for l in lists]
    parts = [torch.stack([kernels.dist_filter(queries[j], sh, N, k, lo, taus[j]) for sh, lo, _ in shards])
             for j in range(a.steps)]
    ps = []
    for j in range(a.steps):
        s_i = [kernels.ip_topk(queries[j], sh, k, id_offset=lo, resolve=True)[:2] for sh, lo, _ in shards]
        ps.append((torch.stack([x[0] for x in s_i]), torch.stack([x[1] for x in s_i])))
    torch.cuda.synchronize()
    own, lo, _ = shards[R]

    if a.check:
        bad = 0
        for j in range(a.steps):
            s1, i1, st = kernels.merge_packed(parts[j], k, N)
            s2, i2 = kernels.topk_merge(ps[j][0], ps[j][1], k)
            bad += int((st != 0).sum()) + int((i1 != i2).any(dim=1).sum())
        out["check_mismatched_queries"] = bad

    fams = {"scan": _native.PROF_SCAN, "sample": _native.PROF_SAMPLE, "select": _native.PROF_SELECT,
            "merge": _native.PROF_MERGE}

    def timed(fn, label, nstreams=1):
        fn(0)
        torch.cuda.synchronize()
        main_s = torch.cuda.current_stream(dev)
        streams = [main_s] + [torch.cuda.Stream(device=dev) for _ in range(nstreams - 1)]
        for f in fams.values():
            lib.drt_profile_enable(f, 1)
        t0 = time.perf_counter()
        for st in streams[1:]:
            st.wait_stream(main_s)
        for j in range(a.steps):
            with torch.cuda.stream(streams[j % len(streams)]):
                fn(j)
        for st in streams[1:]:
            main_s.wait_stream(st)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        res = {"ms_per_step": round(el / a.steps * 1e3, 4)}
        for name, f in fams.items():
            lib.drt_profile_enable(f, 0)
            tot = _native.ctypes.c_double(0.0)
            cnt = _native.c_i64(0)
            lib.drt_profile_read(f, _native.ctypes.byref(tot), _native.ctypes.byref(cnt))
            if cnt.value:
                res[f"{name}_ms"] = round(tot.value / cnt.value, 4)
                res[f"{name}_launches_per_step"] = round(cnt.value / a.steps, 2)
        res["qps_if_comm_free"] = round(qb / (el / a.steps), 1)
        out[label] = res

    # the all-gathers write every rank's slice into one [world, ...] buffer; here rank R's
    # slice is written in place (the other slices hold the precomputed data of the other ranks)
    def gt(j):
        best = kernels.dist_sample(queries[j], own, N, k)
        lists[j][R].copy_(best)
        pk = kernels.dist_filter_lists(queries[j], own, N, k, lo, lists[j])
        parts[j][R].copy_(pk)
        kernels.merge_packed(parts[j], k, N)

    def gt_unfused(j):
        best = kernels.dist_sample(queries[j], own, N, k)
        lists[j][R].copy_(best)
        tau = kernels.dist_tau(lists[j], k)
        pk = kernels.dist_filter(queries[j], own, N, k, lo, tau)
        parts[j][R].copy_(pk)
        kernels.merge_packed(parts[j], k, N)

    def psh(j):
        s, i, _ = kernels.ip_topk(queries[j], own, k, id_offset=lo, resolve=False)
        S, I = ps[j][0].clone(), ps[j][1].clone()
        S[R], I[R] = s, i
        kernels.topk_merge(S, I, k)

    # grouped (search.py _gtau_enqueue_group): one sample launch and one merge per group of
    # G batches, one filter scan per batch
    G = a.group
    groups = [list(range(s0, min(s0 + G, a.steps))) for s0 in range(0, a.steps, G)]
    glists = [torch.cat([lists[j] for j in g], 1).contiguous() for g in groups]
    gparts = [torch.cat([parts[j] for j in g], 1).contiguous() for g in groups]
    gq = [torch.cat([queries[j] for j in g]).contiguous() for g in groups]

    def gt_grouped(gi):
        best = kernels.dist_sample(gq[gi], own, N, k)
        glists[gi][R].copy_(best)
        tau = kernels.dist_tau(glists[gi], k)
        for b, j in enumerate(groups[gi]):
            kernels.dist_filter_into(queries[j], own, N, k, lo, tau[b * qb:(b + 1) * qb],
                                     gparts[gi][R, b * qb:(b + 1) * qb])
        kernels.merge_packed(gparts[gi], k, N)

    def timed_groups(label):
        gt_grouped(0)
        torch.cuda.synchronize()
        for f in fams.values():
            lib.drt_profile_enable(f, 1)
        t0 = time.perf_counter()
        for gi in range(len(groups)):
            gt_grouped(gi)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        res = {"ms_per_step": round(el / a.steps * 1e3, 4), "group_batches": G}
        for name, f in fams.items():
            lib.drt_profile_enable(f, 0)
            tot = _native.ctypes.c_double(0.0)
            cnt = _native.c_i64(0)
            lib.drt_profile_read(f, _native.ctypes.byref(tot), _native.ctypes.byref(cnt))
            if cnt.value:
                res[f"{name}_ms"] = round(tot.value / cnt.value, 4)
                res[f"{name}_launches_per_step"] = round(cnt.value / a.steps, 2)
        res["qps_if_comm_free"] = round(qb / (el / a.steps), 1)
        out[label] = res

    if a.check:
        bad = 0
        for gi, g in enumerate(groups):
            gt_grouped(gi)
            s1, i1, st = kernels.merge_packed(gparts[gi], k, N)
            for b, j in enumerate(g):
                s2, i2 = kernels.topk_merge(ps[j][0], ps[j][1], k)
                sl = slice(b * qb, (b + 1) * qb)
                bad += int((st[sl] != 0).sum()) + int((i1[sl] != i2).any(dim=1).sum())
        out["check_grouped_mismatched_queries"] = bad

    timed_groups("global_tau_grouped")
    timed(gt, "global_tau")
    timed(gt_unfused, "global_tau_unfused")
    timed(psh, "per_shard")
    if a.graph:
        # the rank's compute of one step captured once and replayed: the launch-gap floor
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            gt(0)
        torch.cuda.current_stream(dev).wait_stream(side)
        with torch.cuda.graph(g):
            gt(0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            g.replay()
        torch.cuda.synchronize()
        out["global_tau_graph"] = {"ms_per_step": round((time.perf_counter() - t0) / a.steps * 1e3, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
