"""Patched copies of csrc/search.hip for the round-6 scan32 A/B (not product source)."""
import os, re, sys
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(R, "denseretrievaltoolkits_amd/csrc/search.hip")).read()

OLD_LOOP = """    acc0 = (f32x4){0.f, 0.f, 0.f, 0.f};
    acc1 = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s % RD], qf0[s], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s % RD], qf1[s], acc1, 0, 0, 0);
      // fragment s + RD: of this tile, or (the last RD steps) the first ones of tile it+1
      af[s % RD] = s + RD < KS ? frag(buf, s + RD) : frag(nslot, s + RD - KS);
      __builtin_amdgcn_sched_barrier(0);
      if (s == KS / 4 && do_dma) {
        lt.template issue<false>(a, ring + pslot * C::TILE_BYTES, next_base, ntile == partial_tile, ntile, wave,
                                 lane);
        next_base += tile_stride;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (it > 0) epilogue(prev0, prev1, rb_prev);"""
assert OLD_LOOP in src

def variant(epi_in_gaps, dma_spread):
    lines = ["    acc0 = (f32x4){0.f, 0.f, 0.f, 0.f};",
             "    acc1 = (f32x4){0.f, 0.f, 0.f, 0.f};",
             "    float mx0 = 0.f, mx1 = 0.f;",
             "    bool hit_any = it > 0;",
             "#pragma unroll",
             "    for (int s = 0; s < KS; ++s) {",
             "      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s % RD], qf0[s], acc0, 0, 0, 0);",
             "      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s % RD], qf1[s], acc1, 0, 0, 0);",
             "      af[s % RD] = s + RD < KS ? frag(buf, s + RD) : frag(nslot, s + RD - KS);",
             "      __builtin_amdgcn_sched_barrier(0);"]
    if dma_spread:
        lines += ["      if (do_dma && (s == KS / 4 || s == KS / 4 + 4 || s == KS / 4 + 8)) {",
                  "        lt.issue_one(a, ring + pslot * C::TILE_BYTES, next_base, ntile == partial_tile, ntile, wave, lane,",
                  "                     (s - KS / 4) / 4);",
                  "        if (s == KS / 4 + 8) next_base += tile_stride;",
                  "      }"]
    else:
        lines += ["      if (s == KS / 4 && do_dma) {",
                  "        lt.template issue<false>(a, ring + pslot * C::TILE_BYTES, next_base, ntile == partial_tile, ntile, wave,",
                  "                                 lane);",
                  "        next_base += tile_stride;",
                  "      }"]
    if epi_in_gaps:
        lines += ["      if (s == 2) mx0 = fmaxf(fmaxf(prev0[0], prev0[1]), fmaxf(prev0[2], prev0[3])) - tau0;",
                  "      if (s == 3) mx1 = fmaxf(fmaxf(prev1[0], prev1[1]), fmaxf(prev1[2], prev1[3])) - tau1;",
                  "      if (s == 4) hit_any = hit_any && __ballot(mx0 >= 0.0f || mx1 >= 0.0f) != 0ull;"]
    lines += ["      __builtin_amdgcn_sched_barrier(0);",
              "    }"]
    if epi_in_gaps:
        lines += ["    if (hit_any) epilogue(prev0, prev1, rb_prev);"]
    else:
        lines += ["    if (it > 0) epilogue(prev0, prev1, rb_prev);"]
    return "\n".join(lines)

ISSUE_ONE = """
  // one LDS-DMA piece j of the tile (round-6 A/B: pieces spread over the MFMA chain)
  __device__ __forceinline__ void issue_one(const ScanArgs& a, uint32_t slot_lds, const char* base, bool partial,
                                            int64_t tile, int wave, int lane, int j) {
    if (partial) {
      if (j == 0) issue_tile16<D, NW, false>(a, slot_lds, tile, wave, lane);
      return;
    }
    uint32_t keep;
    const uint32_t vo = j == 0 ? voff[0] : (j == 1 ? voff[G > 1 ? 1 : 0] : voff[G > 2 ? 2 : 0]);
    const uint32_t lo = j == 0 ? loff[0] : (j == 1 ? loff[G > 1 ? 1 : 0] : loff[G > 2 ? 2 : 0]);
    asm volatile(
        "s_mov_b32 %0, m0\\n\\t"
        "s_mov_b32 m0, %2\\n\\t"
        "s_nop 0\\n\\t"
        "global_load_lds_dwordx4 %3, %1\\n\\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "s"(base), "s"(slot_lds + lo), "v"(vo)
        : "memory");
  }
};
"""

for name, e, d in (("e1", True, False), ("e2", False, True), ("e12", True, True)):
    s = src.replace(OLD_LOOP, variant(e, d))
    if d:
        # add issue_one to LeanTile (closing brace of the struct right after the #undef lines)
        anchor = "#undef DRT_LEAN3\n#undef DRT_LEAN1\n  }\n};\n"
        assert anchor in s
        s = s.replace(anchor, "#undef DRT_LEAN3\n#undef DRT_LEAN1\n  }\n" + ISSUE_ONE)
    open(os.path.join(R, f"tools/_ab/search_{name}.hip"), "w").write(s)
    print(name)
