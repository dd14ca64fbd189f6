"""Shared test helpers: seeded synthetic data in the BASELINE layout."""
import numpy as np


def int_bf16(rng, shape, lo=-8, hi=8):
    """Small-integer values: exactly representable in bf16, dot products exact in fp32."""
    return rng.integers(lo, hi + 1, size=shape).astype(np.float32)


def gauss_bf16(rng, shape):
    from oracle.search_oracle import bf16_round
    return bf16_round(rng.standard_normal(shape).astype(np.float32))


def massive_near_ties(n, d, seed=0, nq=2, special=40):
    """(q [nq, d], p [n, d]) bf16-valued fp32 arrays whose n rows share one positive base row (scores
    B ~ 360, fp32 spacing 2^-15) and differ only in a last element below 2^-16, which q's last element (1)
    adds exactly: every exact score is B + t_r, all n inside one fp32 error bound of each other, so a
    near-tie window holds every row (more than the 65,536 the wide resolve / large-k collection take when
    n > 65536).  ``special`` random rows carry the largest tails j 2^-22 (j = 1..special, larger j on a
    smaller id NOT guaranteed), the others random tails below 2^-24: the exact top-k differs from any
    id or fp32 order."""
    from oracle import search_oracle as orc
    rng = np.random.default_rng(seed)
    base = orc.bf16_round(rng.integers(1, 4, size=(1, d)).astype(np.float64) + 0.5)
    p = np.repeat(base, n, axis=0)
    p[:, -1] = orc.bf16_round(rng.random(n) * 2.0 ** -24)
    rows = rng.choice(n, size=special, replace=False)
    p[rows, -1] = np.arange(1, special + 1) * 2.0 ** -22
    q = orc.bf16_round(rng.integers(1, 4, size=(nq, d)).astype(np.float64) + 0.25)
    q[:, -1] = 1.0
    return q.astype(np.float32), p.astype(np.float32)


def to_dev_bf16(x, device):
    import torch
    from oracle.search_oracle import bf16_bits
    t = torch.from_numpy(bf16_bits(x).view(np.int16).copy()).view(torch.bfloat16)
    return t.to(device)


def sample_plan(n, k):
    """Mirror of make_plan() in csrc/search.hip (used only to build adversarial inputs)."""
    import math
    target = max(4096, 4 * k)
    cap = 4 * target
    if n <= cap:
        return None

    def tail(lam, r):
        logp = -lam + r * math.log(lam) - math.lgamma(r + 1.0)
        p = math.exp(logp)
        s = 0.0
        i = r
        while True:
            s += p
            p *= lam / (i + 1)
            i += 1
            if p < 1e-30 * s or i > r + 2000:
                break
        return s

    r = 1
    while tail(k * r / target, r) > 1e-9:
        r += 1
    m = min(n, (r * n + target - 1) // target)
    stride = max(1, n // m)
    m = (n - stride // 2 + stride - 1) // stride
    return dict(r=r, m=m, stride=stride, cap=cap, rows=np.arange(m) * stride + stride // 2)


def corpus_topk_golden():
    """tests/golden/corpus_topk.npz (reference merge_retrieval_results_by_score top-k) plus its
    inputs regenerated from the stored spec (tools/gen_golden.corpus_topk_inputs)."""
    import os
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "corpus_topk.npz"))
    rng = np.random.default_rng(int(z["seed"]))
    lim = int(z["lim"])
    q = rng.integers(-lim, lim + 1, size=(int(z["nq"]), int(z["d"]))).astype(np.float32)
    p = rng.integers(-lim, lim + 1, size=(int(z["n"]), int(z["d"]))).astype(np.float32)
    return q, p, int(z["k"]), int(z["parts"]), z["ids"].astype(np.int64), z["scores"]


def oracle_topk_streamed(q, p_dev, k, chunk=1 << 20, id_offset=0, exact=False):
    """oracle.ip_topk of host queries q [nq, d] over a DEVICE corpus p_dev [n, d] (bf16), streamed to
    the host chunk by chunk (fp32 BLAS: exact for the integer-valued fixtures; ``exact``: fp64, the
    canonical order of real-valued data) and merged with the oracle's partition merge -- the
    full-size reference answer without a full host copy."""
    from oracle.search_oracle import ip_topk, merge_topk
    es = ei = None
    n = p_dev.shape[0]
    for a in range(0, n, chunk):
        if exact:
            pc = p_dev[a: a + chunk].double().cpu().numpy()
            cs, ci = ip_topk(q.astype(np.float64), pc, k, id_offset=id_offset + a, dtype=np.float64,
                             out_dtype=np.float64)
        else:
            pc = p_dev[a: a + chunk].float().cpu().numpy()
            cs, ci = ip_topk(q, pc, k, id_offset=id_offset + a, dtype=np.float32)
        es, ei = (cs, ci) if es is None else merge_topk(np.stack([es, cs]), np.stack([ei, ci]), k)
    return es, ei


def device_int_corpus(n, d, lo, hi, seed, device, chunk=1 << 20):
    """[n, d] bf16 corpus of integers in [lo, hi] generated on the device chunk by chunk (seeded)."""
    import torch
    p = torch.empty((n, d), dtype=torch.bfloat16, device=device)
    g = torch.Generator(device=device).manual_seed(seed)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        p[a:b] = torch.randint(lo, hi + 1, (b - a, d), generator=g, device=device, dtype=torch.int32).to(torch.bfloat16)
    return p
