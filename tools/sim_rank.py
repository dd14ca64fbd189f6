#!/usr/bin/env python3
"""One rank's step of `bench.py --gpus W` on ONE GPU, through the product code itself.

search.ShardedFlatIP.search_batches_iter runs `_gtau_enqueue_group` per group of GROUP_QUERIES queries
(sample, sample-list all-gather, tau, filter, packed all-gather, merge, canonical refine with a delta
all-reduce).  Here every shard of the W-way split lives on this GPU; the other ranks' exchanged
data (sample lists, packed lists) are computed once per group beforehand, and rank R's own
contributions are spliced into those [W, ...] buffers by the `gather` the product calls -- so the
timed region is exactly rank R's device work with the collectives replaced by an in-place copy
(the delta all-reduce by the identity).  Variants (A/B of the filter launch shape):
  group    : the product -- one filter launch over the group's queries (grid corpus tiles x Q/128)
  perbatch : one filter launch per 128-query batch into the same group buffer
usage: python tools/sim_rank.py [--world 8] [--variants group,perbatch] [--batches 32]"""
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
    ap.add_argument("--batches", type=int, default=32)
    ap.add_argument("--variants", default="group,perbatch")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch
    import bench
    from denseretrievaltoolkits_amd import _native, kernels, search as srch
    from denseretrievaltoolkits_amd.search import FlatIPIndex
    lib = _native.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    W, R, k, qb, N = a.world, a.rank, a.k, a.qb, a.n_corpus
    shards = [bench.gen_shard(N, W, r, a.dim, dev) for r in range(W)]
    locs = [FlatIPIndex.from_rows(sh) for sh, _, _ in shards]
    offs = [lo for _, lo, _ in shards]
    st = torch.stack([l.row_stats() for l in locs])
    stats = st.max(0).values.clone()
    stats[1] = st[:, 1].min()   # (ShardedFlatIP.sync_offsets)
    g = torch.Generator(device=dev)
    g.manual_seed(5678)
    queries = [torch.randn((qb, a.dim), generator=g, device=dev).to(torch.bfloat16) for _ in range(a.batches)]
    groups = list(srch._groups(queries))
    kc = kernels.refine_width(k)
    lc = kernels.exchange_cap(kc, W)   # entries per rank list through the exchange (round 6)
    # the other ranks' exchanged data, per group
    glists, gparts = [], []
    for grp in groups:
        qg = torch.cat(grp)
        lists = torch.stack([locs[r].dist_sample(qg, N, k) for r in range(W)]).contiguous()
        tau = kernels.dist_tau(lists, k)
        parts = torch.empty((W, qg.shape[0], lc + 1), dtype=torch.int64, device=dev)
        for r in range(W):
            kernels.dist_filter_into(qg, locs[r].rows, N, lc, offs[r], tau, parts[r])
        glists.append(lists)
        gparts.append(parts)
    torch.cuda.synchronize()
    own, lo = locs[R], offs[R]
    out = {"world": W, "rank": R, "n_corpus": N, "rows_per_rank": int(own.ntotal), "qb": qb, "k": k,
           "batches": a.batches, "group_queries": srch.GROUP_QUERIES, "kc": kc, "exchange_list_entries": lc}
    qg0 = sum(q.shape[0] for q in groups[0])
    r_ = kernels.sample_rank(k)
    # bytes each rank RECEIVES per group through the exchange (the other W - 1 ranks' data): sample lists
    # [Qg, r] u32 + packed lists [Qg, lc + 1] u64 + the canonical stage's delta all-reduce [Qg, kc] f32
    # (a ring all-reduce moves ~2 (W - 1) / W of it through each rank)
    out["exchange_MB_received_per_rank_per_group"] = {
        "sample_lists": round((W - 1) * qg0 * r_ * 4 / 1e6, 2),
        "packed_lists": round((W - 1) * qg0 * (lc + 1) * 8 / 1e6, 2),
        "packed_lists_uncapped": round((W - 1) * qg0 * (kc + 1) * 8 / 1e6, 2),
        "delta_allreduce": round(2 * (W - 1) / W * qg0 * kc * 4 / 1e6, 2)}
    cnt = (gparts[0][:, :, lc] >> 32).float()   # valid entries per (part, query): rows >= tau, capped at lc
    out["hits_per_part"] = {"mean": round(float(cnt.mean()), 1), "min": int(cnt.min()), "max": int(cnt.max()),
                            "full_frac": round(float((cnt >= lc).float().mean()), 4)}

    filt = kernels.dist_filter_into

    def perbatch_filter(q, p, n_global, kk, off, tau, packed):
        for b0 in range(0, q.shape[0], qb):
            filt(q[b0:b0 + qb], p, n_global, kk, off, tau[b0:b0 + qb], packed[b0:b0 + qb])

    fams = {"scan": _native.PROF_SCAN, "sample": _native.PROF_SAMPLE, "select": _native.PROF_SELECT,
            "merge": _native.PROF_MERGE}

    def run_all():
        pend = []
        for gi, grp in enumerate(groups):
            calls = [0]

            def gather(t, gi=gi, calls=calls):
                buf = glists[gi] if calls[0] == 0 else gparts[gi]
                calls[0] += 1
                buf[R].copy_(t)
                return buf
            pend.append(srch._gtau_enqueue_group(own, grp, k, N, lo, gather, stats=stats,
                                                 all_reduce_sum=lambda t: t, world=W))
        nredo = 0
        for p in pend:
            nredo += srch._gtau_finish_group(p, lambda q: (q, q))[1]
        run_all.redone = nredo

    for rep in range(a.reps):
        for var in a.variants.split(","):
            kernels.dist_filter_into = perbatch_filter if var == "perbatch" else filt
            run_all()
            torch.cuda.synchronize()
            for f in fams.values():
                lib.drt_profile_enable(f, 1)
            t0 = time.perf_counter()
            run_all()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            res = {"rep": rep, "variant": var, "batches_uncertified": run_all.redone,
                   "ms_per_batch": round(el / a.batches * 1e3, 4),
                   "qps_if_comm_free": round(a.batches * qb / el, 1)}
            for name, f in fams.items():
                lib.drt_profile_enable(f, 0)
                tot = _native.ctypes.c_double(0.0)
                cnt = _native.c_i64(0)
                lib.drt_profile_read(f, _native.ctypes.byref(tot), _native.ctypes.byref(cnt))
                if cnt.value:
                    res[f"{name}_ms_per_launch"] = round(tot.value / cnt.value, 4)
                    res[f"{name}_ms_per_batch"] = round(tot.value / a.batches, 4)
            print(json.dumps(res), flush=True)
    kernels.dist_filter_into = filt
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
