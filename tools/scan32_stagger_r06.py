"""Patched copy of csrc/search.hip for the round-6 scan32 stagger A/B (not product source):
waves NW/2.. run half a tile AHEAD of waves 0..NW/2-1 (MI355X_MICROARCH.md 'Two waves per SIMD' item 9),
so each SIMD's two waves reach their hit-check epilogue and barrier wait at different points of the
MFMA stream.  Same ring protocol (at barrier it every wave is past tile it-1; the upper half reads
only tiles it and it+1 in window it), same barrier count, same MFMA chain per tile: outputs identical.
usage: python tools/scan32_stagger_r06.py [EP]  ->  tools/_ab/search_stg.hip"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(R, "denseretrievaltoolkits_amd/csrc/search.hip")).read()
EP = int(sys.argv[1]) if len(sys.argv) > 1 else 4

OLD = """  f32x4 a0, a1, b0, b1;
  uint32_t rbA = 0, rbB = 0;
  for (int it = 0; it < my_tiles; it += 2) {
    iter(it, a0, a1, rbA, b0, b1, rbB);
    if (it + 1 < my_tiles) iter(it + 1, b0, b1, rbB, a0, a1, rbA);
  }
  if (my_tiles & 1) epilogue(a0, a1, rbA);
  else epilogue(b0, b1, rbB);
  if (wcnt) wave_flush_hits(a, qw, hk, hq, wcnt, lane);
}"""
assert src.count(OLD) == 1

NEW = """  f32x4 a0, a1, b0, b1;
  uint32_t rbA = 0, rbB = 0;
  constexpr int KH = KS / 2;
  constexpr int EP0 = %d;   // k-steps of the next tile issued before the upper half's deferred epilogue
  constexpr int EP = EP0 < KH ? EP0 : KH;
  constexpr bool STG = KS %% 2 == 0 && KH + RD <= KS && KS >= 8;   // d >= 256
  // upper half: window it = tile it's second half, then tile it+1's first half (the epilogue of tile it
  // after EP k-steps of tile it+1)
  auto riter = [&](int it, f32x4& c0, f32x4& c1, f32x4& n0, f32x4& n1) {
    const int tile = t0 + it * tstep;
    if (it + PD <= my_tiles) {
      wait_vmcnt<C::GLDS_PER_WAVE * (PD - 2)>();
    } else if (it + 1 < my_tiles) {
      wait_tiles_younger<C::GLDS_PER_WAVE>(my_tiles - 1 - it - 1);
    }
    lds_barrier();
    const bool do_dma = it + PD < my_tiles;
    const int ntile = tile + PD * tstep;
    const int pslot = buf == 0 ? NB - 1 : buf - 1;
    const int nslot = buf + 1 == NB ? 0 : buf + 1;
#pragma unroll
    for (int s = KH; s < KS; ++s) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s %% RD], qf0[s], c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s %% RD], qf1[s], c1, 0, 0, 0);
      af[s %% RD] = s + RD < KS ? frag(buf, s + RD) : frag(nslot, s + RD - KS);
      __builtin_amdgcn_sched_barrier(0);
      if (s == KH + KS / 4 && do_dma) {
        lt.template issue<false>(a, ring + pslot * C::TILE_BYTES, next_base, ntile == partial_tile, ntile, wave,
                                 lane);
        next_base += tile_stride;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    const uint32_t rb = (uint32_t)tile * kT16 + 4 * kq;
    if (it + 1 < my_tiles) {
      n0 = (f32x4){0.f, 0.f, 0.f, 0.f};
      n1 = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KH; ++s) {
        n0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s %% RD], qf0[s], n0, 0, 0, 0);
        n1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s %% RD], qf1[s], n1, 0, 0, 0);
        af[s %% RD] = frag(nslot, s + RD);
        __builtin_amdgcn_sched_barrier(0);
        if (s == EP - 1) epilogue(c0, c1, rb);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      epilogue(c0, c1, rb);
    }
    buf = nslot;
  };
  if (STG && wave >= NW / 2) {
    // pre-step: tile 0's first half (tile 0 landed at the prologue barrier)
    a0 = (f32x4){0.f, 0.f, 0.f, 0.f};
    a1 = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KH; ++s) {
      a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s %% RD], qf0[s], a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s %% RD], qf1[s], a1, 0, 0, 0);
      af[s %% RD] = frag(0, s + RD);
      __builtin_amdgcn_sched_barrier(0);
    }
    for (int it = 0; it < my_tiles; it += 2) {
      riter(it, a0, a1, b0, b1);
      if (it + 1 < my_tiles) riter(it + 1, b0, b1, a0, a1);
    }
  } else {
    for (int it = 0; it < my_tiles; it += 2) {
      iter(it, a0, a1, rbA, b0, b1, rbB);
      if (it + 1 < my_tiles) iter(it + 1, b0, b1, rbB, a0, a1, rbA);
    }
    if (my_tiles & 1) epilogue(a0, a1, rbA);
    else epilogue(b0, b1, rbB);
  }
  if (wcnt) wave_flush_hits(a, qw, hk, hq, wcnt, lane);
}""" % EP

s = src.replace(OLD, NEW)
os.makedirs(os.path.join(R, "tools/_ab"), exist_ok=True)
out = os.path.join(R, f"tools/_ab/search_stg{EP}.hip")
open(out, "w").write(s)
print(out)
