"""What v_mfma_f32_16x16x32_bf16 computes, bit for bit (diagnostic for the canonical-order bound).

Runs tools/mfma_numerics.hip (built to tools/mfma_numerics.so by tools/build_probe.sh) on seeded
inputs and compares every output with candidate summation models of D = C + sum_k a_k b_k:
  exact_rn   the exact sum rounded once to fp32 (nearest even)
  exact_rz   ... rounded once toward zero
  seq_rn     C, then the 32 products added one by one in k order, each add rounded (fp32 fma chain)
  tree_rn    the 32 products summed pairwise in fp32, then + C
Then chains of S = 24 steps (d = 768, the scan's accumulation) against the per-step models, and the
worst error of the hardware chain against the exact sum, in units of u * sum |a b| (u = 2^-24) and of
u * sum_t |partial sum t| -- the quantities the bound of csrc/search.hip refine_eps is built from.
Prints one JSON object.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def bf16(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return u


def from_bf16(u):
    return (u.astype(np.uint32) << 16).view(np.float32)


def run(lib, A, B, C, fn="mfma_chain"):
    T, S = A.shape[0], A.shape[1]
    dev = torch.device("cuda", 0)
    a = torch.from_numpy(A.view(np.int16).copy()).to(dev)
    b = torch.from_numpy(B.view(np.int16).copy()).to(dev)
    c = torch.from_numpy(C.astype(np.float32)).to(dev)
    d = torch.empty_like(c)
    s = torch.cuda.current_stream().cuda_stream
    rc = getattr(lib, fn)(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(c.data_ptr()),
                        ctypes.c_void_p(d.data_ptr()), T, S, ctypes.c_void_p(s))
    assert rc == 0, rc
    torch.cuda.synchronize()
    return d.cpu().numpy()


def rz32(x):
    f = x.astype(np.float32)
    over = np.abs(f.astype(np.float64)) > np.abs(x)
    f[over] = np.nextafter(f[over], np.float32(0))
    return f


def products(A, B):
    """[T, S, 16 m, 16 n, 32 k] exact products (fp64)."""
    a = from_bf16(A).astype(np.float64)
    b = from_bf16(B).astype(np.float64)
    return a[:, :, :, None, :] * b[:, :, None, :, :]


def step_models(C, P):
    """One step: C [T,16,16] fp32, P [T,16,16,32] fp64 exact products -> dict of model outputs."""
    ex = C.astype(np.float64) + P.sum(-1)   # exact for the magnitudes used here (<= 53 bits)
    out = {"exact_rn": ex.astype(np.float32), "exact_rz": rz32(ex)}
    acc = C.astype(np.float32)
    for k in range(32):
        acc = (acc.astype(np.float64) + P[..., k]).astype(np.float32)
    out["seq_rn"] = acc
    v = P.astype(np.float32)
    while v.shape[-1] > 1:
        v = v[..., 0::2] + v[..., 1::2]
    out["tree_rn"] = (C.astype(np.float32) + v[..., 0]).astype(np.float32)
    return out


def one_step(lib, rng, T, gen_ab, gen_c):
    A = bf16(gen_ab((T, 1, 16, 32)))
    B = bf16(gen_ab((T, 1, 16, 32)))
    C = gen_c((T, 16, 16)).astype(np.float32)
    D = run(lib, A, B, C)
    P = products(A, B)[:, 0]
    r = {m: float((D == v).mean()) for m, v in step_models(C, P).items()}
    ex = C.astype(np.float64) + P.sum(-1)
    err = np.abs(D.astype(np.float64) - ex)
    u = 2.0 ** -24
    r["err_over_u_exact"] = float((err / (u * np.abs(ex) + 1e-300)).max())
    r["err_over_u_c_plus_abs"] = float((err / (u * (np.abs(C) + np.abs(P).sum(-1)) + 1e-300)).max())
    r["err_over_u_max_term"] = float((err / (u * np.maximum(np.abs(C), np.abs(P).max(-1)) + 1e-300)).max())
    return r


def chain(lib, rng, T, S, gen_ab):
    A = bf16(gen_ab((T, S, 16, 32)))
    B = bf16(gen_ab((T, S, 16, 32)))
    C = np.zeros((T, 16, 16), np.float32)
    D = run(lib, A, B, C).astype(np.float64)
    P = products(A, B)                                   # [T,S,16,16,32]
    ps = P.sum(-1)                                       # per-step exact sums
    exact = ps.sum(1)
    absum = np.abs(P).sum((1, -1))
    partial = np.abs(np.cumsum(ps, axis=1)).sum(1)       # sum_t |exact partial sum after step t|
    accs = {}
    for m in ("exact_rn", "exact_rz", "seq_rn"):
        acc = C.copy()
        for s in range(S):
            acc = step_models(acc, P[:, s])[m]
        accs[m] = float((acc == D.astype(np.float32)).mean())
    u = 2.0 ** -24
    err = np.abs(D - exact)
    return {
        "match": accs,
        "max_err_over_u_abssum": float((err / (u * absum + 1e-300)).max()),
        "max_err_over_u_partials": float((err / (u * partial + 1e-300)).max()),
        "max_err_over_u_norms": float((err / (u * np.sqrt((from_bf16(A).astype(np.float64) ** 2).sum((1, 3)))[:, :, None]
                                               * np.sqrt((from_bf16(B).astype(np.float64) ** 2).sum((1, 3)))[:, None, :]
                                               + 1e-300)).max()),
    }


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "mfma_numerics.so"))
    rng = np.random.default_rng(0)
    out = {}
    g = lambda sh: rng.standard_normal(sh)
    out["gauss_c0"] = one_step(lib, rng, 2048, g, lambda sh: np.zeros(sh))
    out["gauss_c_big"] = one_step(lib, rng, 2048, g, lambda sh: 1e3 * rng.standard_normal(sh))
    out["gauss_c_tiny"] = one_step(lib, rng, 2048, g, lambda sh: 1e-3 * rng.standard_normal(sh))
    # wide exponent spread inside one step (cancellation): scales 2^-8 .. 2^8 per element
    w = lambda sh: rng.standard_normal(sh) * np.exp2(rng.integers(-8, 9, size=sh))
    out["spread_c0"] = one_step(lib, rng, 2048, w, lambda sh: np.zeros(sh))
    out["spread_c"] = one_step(lib, rng, 2048, w, lambda sh: 30.0 * rng.standard_normal(sh))
    # positive near-degenerate products (the C2 tower's regime): large common part, tiny rest
    pos = lambda sh: 1.0 + 1e-2 * rng.standard_normal(sh)
    out["positive_c"] = one_step(lib, rng, 2048, pos, lambda sh: 500.0 + rng.standard_normal(sh))
    # one dominant product and 31 tiny ones of mixed sign (alignment truncation shows as bias)
    def dom(sh):
        x = 1e-3 * rng.standard_normal(sh)
        x[..., 0] = 8.0
        return x
    out["dominant_c0"] = one_step(lib, rng, 2048, dom, lambda sh: np.zeros(sh))
    out["dominant_c"] = one_step(lib, rng, 2048, dom, lambda sh: 100.0 * rng.standard_normal(sh))
    # all-positive products over 30 binades below the largest: truncated alignment loses the most here
    ps = lambda sh: np.exp2(-rng.uniform(0, 30, size=sh))
    out["pos_spread_c0"] = one_step(lib, rng, 4096, ps, lambda sh: np.zeros(sh))
    out["pos_spread_c"] = one_step(lib, rng, 4096, ps, lambda sh: np.abs(rng.standard_normal(sh)))
    ps2 = lambda sh: np.exp2(-rng.uniform(10, 14, size=sh)) * (1 + (np.arange(sh[-1]) == 0) * 2 ** 12)
    out["pos_one_big_c0"] = one_step(lib, rng, 4096, ps2, lambda sh: np.zeros(sh))
    out["tiny_vs_c"] = one_step(lib, rng, 2048, g, lambda sh: 1e6 * rng.standard_normal(sh))
    # C = 2^24 and products 1: sequential adds lose every 1 (ties to even), one rounding keeps them
    A = np.full((1, 1, 16, 32), 0x3F80, np.uint16)
    D = run(lib, A, A.copy(), np.full((1, 16, 16), 2.0 ** 24, np.float32))
    out["c_2p24_plus_32_ones"] = float(D[0, 0, 0] - 2.0 ** 24)
    # alignment: one product 1 (or C = 1) and 31 (32) equal positive products 2^-j: how much of their
    # sum survives, in units of 2^-24 (= u * 1); sequential RN keeps 0 below j = 24, an exact sum all
    def small_terms(j, in_c):
        A = np.full((1, 1, 16, 32), bf16(np.float32(2.0 ** -j))[()], np.uint16)
        Bm = np.full((1, 1, 16, 32), 0x3F80, np.uint16)
        C = np.zeros((1, 16, 16), np.float32)
        if in_c:
            C[:] = 1.0
            nsmall = 32
        else:
            A[..., 0] = 0x3F80
            nsmall = 31
        D = run(lib, A, Bm, C)
        return {"kept_units_2m24": float((D[0, 0, 0].astype(np.float64) - 1.0) / 2.0 ** -24),
                "exact_units_2m24": nsmall * 2.0 ** (24 - j)}
    out["align_product"] = {j: small_terms(j, False) for j in range(20, 33, 2)}
    out["align_c"] = {j: small_terms(j, True) for j in range(20, 33, 2)}
    # mixed signs around the alignment cut: +1, then 31 products of -2^-j (borrow behaviour)
    def neg_terms(j):
        A = np.full((1, 1, 16, 32), bf16(np.float32(-(2.0 ** -j)))[()], np.uint16)
        A[..., 0] = 0x3F80
        Bm = np.full((1, 1, 16, 32), 0x3F80, np.uint16)
        D = run(lib, A, Bm, np.zeros((1, 16, 16), np.float32))
        return {"got_minus_1_units_2m24": float((D[0, 0, 0].astype(np.float64) - 1.0) / 2.0 ** -24),
                "exact_units_2m24": -31 * 2.0 ** (24 - j)}
    out["align_negative"] = {j: neg_terms(j) for j in range(20, 33, 2)}
    out["chain24_gauss"] = chain(lib, rng, 512, 24, g)
    out["chain24_positive"] = chain(lib, rng, 512, 24, pos)
    out["chain24_spread"] = chain(lib, rng, 512, 24, w)
    # adversarial: large cancelling pairs across steps + small rest
    def adv(sh):
        x = 1e-2 * rng.standard_normal(sh)
        x[..., 0] = 64.0 * np.sign(rng.standard_normal(sh[:-1]))
        return x
    out["chain24_cancel"] = chain(lib, rng, 512, 24, adv)
    # v_mfma_f32_32x32x16_bf16 (the grouped filter scan): 16 products per step
    def one_step32(gen_ab, gen_c, T=512):
        A = bf16(gen_ab((T, 1, 32, 16)))
        B = bf16(gen_ab((T, 1, 32, 16)))
        C = gen_c((T, 32, 32)).astype(np.float32)
        D = run(lib, A, B, C, "mfma32_chain")
        P = products(A, B)[:, 0]
        ex = C.astype(np.float64) + P.sum(-1)
        err = np.abs(D.astype(np.float64) - ex)
        u = 2.0 ** -24
        return {"exact_rn_match": float((D == ex.astype(np.float32)).mean()),
                "err_over_u_c_plus_abs": float((err / (u * (np.abs(C) + np.abs(P).sum(-1)) + 1e-300)).max())}
    out["mm32_gauss_c0"] = one_step32(g, lambda sh: np.zeros(sh))
    out["mm32_spread_c"] = one_step32(w, lambda sh: 30.0 * rng.standard_normal(sh))
    out["mm32_pos_one_big"] = one_step32(ps2, lambda sh: np.zeros(sh))
    out["mm32_dominant_c"] = one_step32(dom, lambda sh: 100.0 * rng.standard_normal(sh))
    def ones_in_c(j):
        A = np.full((1, 1, 32, 16), bf16(np.float32(2.0 ** -j))[()], np.uint16)
        Bm = np.full((1, 1, 32, 16), 0x3F80, np.uint16)
        D = run(lib, A, Bm, np.ones((1, 32, 32), np.float32), "mfma32_chain")
        return float((D[0, 0, 0].astype(np.float64) - 1.0) / 2.0 ** -24)
    out["mm32_align_c_units_2m24"] = {j: ones_in_c(j) for j in (22, 24, 26, 27, 28)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    sys.exit(main())
