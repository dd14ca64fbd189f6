"""Patched copy of csrc/gemm.hip for the round-6 A/B of a PERSISTENT pr5 whose epilogue stores drain
under the next tile's MFMA loop (not product source until it wins):
  * grid = one round of work-groups, each looping over the tiles v = bid, bid + grid, ... (the same
    XCD-remapped tile order as pr5's one-tile work-groups);
  * the ring's LDS-DMA is issued by group 0 (waves 0-3) alone, 8 per wave per memory segment, and only
    group 0 waits on vmcnt;
  * at a tile's end every wave stages its bf16 outputs in LDS (slots 0-3) while group 0 already streams the
    next tile's X_0 into slot 4; group 1 then reads all 128 KiB back and issues every global store.  Group 1
    never waits on vmcnt, so the stores drain while the next tile's MFMAs run (pr5's burst of every CU
    writing its tile at once is what the r05 ablation priced at 20-31 % of each GEMM);
  * same MFMA chains per output element: outputs bit-identical to pr5.
Inference epilogues only (bf16 out, BIAS or BIAS | GELU, full 256-column tiles, no split-K).
usage: python tools/gemm_pr5p_r06.py -> tools/_ab/gemm_pr5p.hip"""
import os

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(R, "denseretrievaltoolkits_amd/csrc/gemm.hip")).read()

KERNEL = r'''
// ---- round-6 A/B: persistent pr5, group 0 loads, group 1 stores (tools/gemm_pr5p_r06.py) ----
__device__ __forceinline__ void stage_panel64_g0(const __bf16* base, int64_t ld, int64_t row0, int64_t rows,
                                                 int64_t k0, uint32_t lds, int wave, int lane, int lane_off) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int J = j * 4 + wave;           // 0..31, waves 0..3
    const int64_t r = row0 + J * 8;
    const char* p = (const char*)(base + r * ld + k0);
    int off = lane_off;
    if (r + 8 > rows) {
      const int rsub = lane >> 3;
      const int64_t gr = r + rsub < rows ? r + rsub : rows - 1;
      off = (int)((gr - r) * ld * 2) + (((lane & 7) ^ rsub) << 4);
    }
    g_glds16(p + off, __builtin_amdgcn_readfirstlane(lds + J * 1024));
  }
}

template <int EPI>
__global__ __launch_bounds__(kLThreads, 1) void gemm_nt_pr5p_kernel(GemmArgs a, int ntiles) {
  __shared__ __attribute__((aligned(16))) char smem[5 * kQPanel];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int grp = wave >> 2;
  const int wn = wave & 3;
  const int nwg = gridDim.x;
  const int tiles_n = (int)((a.n + kL - 1) / kL);
  const int nt = (int)(a.k / 64);
  const uint32_t lds0 = g_lds_addr(smem);
  const int fr = lane & 15, fc = lane >> 4;
  const int foff0 = fr * 128 + ((fc ^ (fr & 7)) << 4);
  const int foff1 = fr * 128 + (((4 + fc) ^ (fr & 7)) << 4);
  const int loffA = panel64_lane_off(a.lda, lane), loffB = panel64_lane_off(a.ldb, lane);
  const int xrow = grp * 128 * 128;
  const int wrow = wn * 64 * 128;
  auto tile_of = [&](int v, int64_t& m0, int64_t& n0) {
    const int xcd = v & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (v >> 3);
    int tm, tn;
    tile_order(a.order, wg, ntiles, tiles_n, tm, tn);
    m0 = (int64_t)tm * kL;
    n0 = (int64_t)tn * kL;
  };
  auto stage_x = [&](int64_t m0, int t, int slot) {
    stage_panel64_g0(a.A, a.lda, m0, a.m, (int64_t)t * 64, lds0 + slot * kQPanel, wave, lane, loffA);
  };
  auto stage_w = [&](int64_t n0, int t, int slot) {
    stage_panel64_g0(a.B, a.ldb, n0, a.n, (int64_t)t * 64, lds0 + slot * kQPanel, wave, lane, loffB);
  };

  int v = blockIdx.x;
  int64_t m0, n0;
  tile_of(v, m0, n0);
  // prologue of the first tile: X_0 (slot 4), W_0 (slot 0) landed, X_1 (slot 1) in flight
  if (grp == 0) {
    stage_x(m0, 0, 4);
    stage_w(n0, 0, 0);
    if (nt > 1) {
      stage_x(m0, 1, 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  for (;;) {
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int xs = 4;   // slot of X_t = (4 + 2t) mod 5; W_t in xs + 1 (mod 5)
    for (int t = 0; t < nt; ++t) {
      const int ws = xs == 4 ? 0 : xs + 1;
      const char* X = smem + xs * kQPanel + xrow;
      const char* W = smem + ws * kQPanel + wrow;
      bf16x8 wf[4], xf[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) wf[j] = *(const bf16x8*)(W + j * 16 * 128 + foff0);
#pragma unroll
      for (int i = 0; i < 8; ++i) xf[i] = *(const bf16x8*)(X + i * 16 * 128 + foff0);
      if (grp == 0 && t + 1 < nt) stage_w(n0, t + 1, xs + 3 >= 5 ? xs - 2 : xs + 3);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int j = 0; j < 4; ++j) wf[j] = *(const bf16x8*)(W + j * 16 * 128 + foff1);
#pragma unroll
      for (int i = 0; i < 8; ++i) xf[i] = *(const bf16x8*)(X + i * 16 * 128 + foff1);
      if (grp == 0) {
        if (t + 2 < nt) {
          stage_x(m0, t + 2, xs + 4 >= 5 ? xs - 1 : xs + 4);
          asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      xs = xs + 2 >= 5 ? xs - 3 : xs + 2;
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();   // every wave past group 1's last MFMA segment: all slots free
    __builtin_amdgcn_sched_barrier(0);
    const int vn = v + nwg;
    const bool has_next = vn < ntiles;
    int64_t m1 = 0, n1 = 0;
    if (has_next) tile_of(vn, m1, n1);
    if (has_next && grp == 0) stage_x(m1, 0, 4);   // the next tile's X_0 under this tile's epilogue
    // every wave: bias (+ GELU) -> bf16 -> its own 16 KiB staging region (slots 0-3), [128 rows][8 x 16 B]
    {
      char* lds_wave = smem + wave * 16384;
      const int64_t colw = n0 + wn * 64;
      f32x4 bv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = *(const f32x4*)(a.bias + colw + j * 16 + 4 * fc);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = i * 16 + fr;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bf16x4 o;
#pragma unroll
          for (int u = 0; u < 4; u += 2) {
            f32x2 x = {acc[i][j][u] * a.alpha + bv[j][u], acc[i][j][u + 1] * a.alpha + bv[j][u + 1]};
            if (EPI & EPI_GELU) x = gelu_fast2(x);
            o[u] = (__bf16)x.x;
            o[u + 1] = (__bf16)x.y;
          }
          const int chunk = (2 * j + (fc >> 1)) ^ (r & 7);
          *(bf16x4*)(lds_wave + r * 128 + chunk * 16 + (fc & 1) * 8) = o;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (grp == 1) {   // group 1 stores the whole tile: regions of waves wn (rows 0-127) and 4 + wn (128-255)
      const int c = lane & 7;
      const int64_t colw = n0 + wn * 64;
#pragma unroll 1
      for (int q = 0; q < 8; ++q) {   // 4 rows of 16 B per lane per step: 16 VGPRs in flight
        const int h = q >> 2;
        const char* reg = smem + (h * 4 + wn) * 16384;
        bf16x8 val[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = ((q & 3) * 4 + u) * 8 + (lane >> 3);
          val[u] = *(const bf16x8*)(reg + r * 128 + ((c ^ (r & 7)) << 4));
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = ((q & 3) * 4 + u) * 8 + (lane >> 3);
          const int64_t row = m0 + h * 128 + r;
          if (row < a.m) __builtin_nontemporal_store(val[u], (bf16x8*)((__bf16*)a.C + row * a.ldc + colw + c * 8));
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();   // staging read back: slots 0-3 free
    __builtin_amdgcn_sched_barrier(0);
    if (!has_next) break;
    if (grp == 0) {
      stage_w(n1, 0, 0);
      if (nt > 1) {
        stage_x(m1, 1, 1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __builtin_amdgcn_s_barrier();
    if (grp == 1) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    v = vn;
    m0 = m1;
    n0 = n1;
  }
}
'''

anchor = "static int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }"
assert src.count(anchor) == 1
src = src.replace(anchor, KERNEL + "\n" + anchor)

old_launch = """    case GP_LARGE:
      // whole-line K-tiles in the 5-slot panel ring (tools/gemm_ab.py: +5-18 % over the 32-deep
      // slab ring, bit-identical outputs)
      hipLaunchKernelGGL((gemm_nt_pr5_kernel<OUT_BF16, EPI>), dim3((unsigned)tiles_l), dim3(kLThreads), 0, s, a);
      break;"""
assert src.count(old_launch) == 1
new_launch = """    case GP_LARGE:
      if constexpr (OUT_BF16 && (EPI == EPI_BIAS || EPI == (EPI_BIAS | EPI_GELU))) {
        if (a.n % kL == 0 && a.ldc % 8 == 0 && a.k % 64 == 0 && a.bias != nullptr) {
          const int64_t cus = gemm_cus() / 8 * 8;
          const int64_t g = tiles_l < cus ? tiles_l : cus;
          hipLaunchKernelGGL((gemm_nt_pr5p_kernel<EPI>), dim3((unsigned)g), dim3(kLThreads), 0, s, a, (int)tiles_l);
          break;
        }
      }
      hipLaunchKernelGGL((gemm_nt_pr5_kernel<OUT_BF16, EPI>), dim3((unsigned)tiles_l), dim3(kLThreads), 0, s, a);
      break;"""
src = src.replace(old_launch, new_launch)
os.makedirs(os.path.join(R, "tools/_ab"), exist_ok=True)
out = os.path.join(R, "tools/_ab/gemm_pr5p.hip")
open(out, "w").write(src)
print(out)
