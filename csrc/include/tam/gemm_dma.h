// tiresias_amd — LDS-DMA pipelined GEMM for the small/medium shapes of the
// model zoo (Transformer-base linears M=4096 x N=512..2048 x K=512..2048, the
// GNMT LSTM recurrence M=64 x N=4096 x K=1024, ResNet 1x1 convs), all four
// operand majorities:
//
//   C[M][N] (op)= alpha * sum_k A(m,k) B(k,n)   bf16 in, fp32 accumulate
//   A(m,k) = AK ? A[m*lda + k] : A[k*lda + m]     B(k,n) = BK ? B[n*ldb + k] : B[k*ldb + n]
//
// Why: the register-staged 64x64 igemm spends these shapes waiting on
// global-load latency (one K-tile in flight, ~20 us for a 2-GFLOP GEMM whose
// bytes and FLOPs take ~3 us). Here every K-tile (BK = 64) of both operands
// goes HBM/L2 -> LDS with global_load_lds_dwordx4 into a STAGES-deep ring, so
// STAGES-1 tiles are in flight while one is multiplied; one raw barrier per
// K-tile with a counted vmcnt (the pipeline never drains inside the loop).
// LDS images (the XOR swizzles of igemm.h applied on the DMA source chunk):
//   K-major operand : [rows][64] bf16, fragments by ds_read_b128 (read_frag_k)
//   MN-major operand: [64 k][<=128 cols] sub-images, fragments by the
//                     transposing ds_read_b64_tr_b16 (read_frag_mn)
// bf16 outputs leave through a per-wave LDS slab as 16-B row chunks (bias,
// ReLU, relu-backward mask, accumulate fused); fp32 outputs store / add /
// atomically add (split-K) in the MFMA C layout.
// Requirements (host checks): K % 64 == 0; MN-major operands need their
// M (or N) % 8 == 0; leading dims % 8 == 0; 16-B aligned bases.
#pragma once
#include "tam/conv_dma.h"
#include "tam/tiles.h"

namespace tam {

struct GDArgs {
  const bf16_t* A;
  long lda;
  const bf16_t* B;
  long ldb;
  int M, N, K;
  int kps;   // K-tiles per split (blockIdx.z)
};

template <int S>
__device__ __forceinline__ int gd_swz16(int row) { return mnmaj_swz<S>(row) >> 1; }

// one operand's per-thread DMA plan. K-major: instruction g covers rows
// 8g..8g+7 (lane -> row lane/8, 16-B chunk lane%8). MN-major: sub-image
// h = g / (S/8) of S columns, instruction li covers k-rows RPI*li.. (lane ->
// k-row lane/(S/8), chunk lane%(S/8)).
template <int EXT, bool KMAJ, int W>
struct GdOperand {
  static constexpr int I = EXT / 8 / W;            // DMA instructions per thread per K-tile
  static constexpr int S = EXT < 128 ? EXT : 128;  // MN-major sub-image width
  static constexpr int BYTES = EXT * 64 * 2;
  const bf16_t* ptr[I];
  int krow[I];                                      // MN-major: k-row of the lane's slot
  __device__ void init(const bf16_t* base, long ld, int extent, int e0, int wid, int lane) {
#pragma unroll
    for (int j = 0; j < I; ++j) {
      const int g = wid + W * j;
      if constexpr (KMAJ) {
        const int r = g * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        int row = e0 + r;
        row = row < extent ? row : extent - 1;      // rows past the edge are never stored
        ptr[j] = base + (long)row * ld + c * 8;
        krow[j] = 0;
      } else {
        constexpr int LPR = S / 8, RPI = 64 / LPR;
        const int h = g / (S / 8), li = g % (S / 8);
        const int kr = RPI * li + lane / LPR;
        const int c = (lane % LPR) ^ gd_swz16<S>(kr);
        int col = e0 + h * S + 8 * c;
        col = col + 8 <= extent ? col : extent - 8;   // chunks past the edge are never stored
        ptr[j] = base + (long)kr * ld + col;
        krow[j] = kr;
      }
    }
  }
  __device__ void issue(char* tile, long ld, int k0, int wid) const {
#pragma unroll
    for (int j = 0; j < I; ++j) {
      const int g = wid + W * j;
      const bf16_t* p = KMAJ ? ptr[j] + k0 : ptr[j] + (long)k0 * ld;
      char* dst;
      if constexpr (KMAJ) dst = tile + g * 1024;
      else dst = tile + (g / (S / 8)) * (64 * S * 2) + (g % (S / 8)) * 1024;
      __builtin_amdgcn_global_load_lds((const void*)p, (cd_lds_void_t*)dst, 16, 0, 0);
    }
  }
  // fragment of 16 rows/cols starting at `base` of the tile, k-half kk
  __device__ static s16x8_t frag(const char* tile, int lane, int base, int kk) {
    if constexpr (KMAJ) return read_frag_k(tile, lane, base, kk);
    else return read_frag_mn<S>(tile + (base / S) * (64 * S * 2), lane, 32 * kk, base % S);
  }
};

template <int BM, int BN, int WM, int WN, bool AK, bool BKM, int STAGES>
__global__ void __launch_bounds__(64 * WM * WN) gemm_dma_kernel(GDArgs a, Epi ep) {
  constexpr int W = WM * WN, BK = 64;
  using OA = GdOperand<BM, AK, W>;
  using OB = GdOperand<BN, BKM, W>;
  static_assert(OA::I >= 1 && OB::I >= 1 && BM % (8 * W) == 0 && BN % (8 * W) == 0, "wave split");
  constexpr int STAGE = OA::BYTES + OB::BYTES;
  constexpr int D = OA::I + OB::I;
  constexpr int WROWS = BM / WM, WCOLS = BN / WN;
  constexpr int TM = WROWS / 16, TN = WCOLS / 16;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % WM, wn = wid / WM;
  const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int grp = bid / per_group;
  const int first_m = grp * GROUP;
  const int gsize = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (bid % per_group) % gsize;
  const int tn = (bid % per_group) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  const int ktiles = a.K / BK;
  const int kt0 = blockIdx.z * a.kps;
  const int nk = min(ktiles - kt0, a.kps);

  OA oa;
  OB ob;
  oa.init(a.A, a.lda, a.M, m0, wid, lane);
  ob.init(a.B, a.ldb, a.N, n0, wid, lane);

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int t, int st) {
    char* sa = smem + st * STAGE;
    oa.issue(sa, a.lda, (kt0 + t) * BK, wid);
    ob.issue(sa + OA::BYTES, a.ldb, (kt0 + t) * BK, wid);
  };

  if (nk > 0) {
#pragma unroll
    for (int t = 0; t < STAGES - 1; ++t)
      if (t < nk) issue(t, t);
    for (int t = 0; t < nk; ++t) {
      // retire tile t: the younger min(STAGES-2, nk-1-t) tiles stay in flight
      const int ahead = min(STAGES - 2, nk - 1 - t);
      if constexpr (STAGES >= 4) {
        if (ahead >= 2) cd_vm_wait<2 * D>();
        else if (ahead == 1) cd_vm_wait<D>();
        else cd_vm_wait<0>();
      } else if constexpr (STAGES == 3) {
        if (ahead >= 1) cd_vm_wait<D>();
        else cd_vm_wait<0>();
      } else {
        cd_vm_wait<0>();
      }
      cd_barrier();
      if (t + STAGES - 1 < nk) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
      const char* ta = smem + (t % STAGES) * STAGE;
      const char* tb = ta + OA::BYTES;
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        s16x8_t fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = OA::frag(ta, lane, wm * WROWS + 16 * i, kk);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = OB::frag(tb, lane, wn * WCOLS + 16 * j, kk);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8_t, fa[i]), __builtin_bit_cast(bf16x8_t, fb[j]), acc[i][j],
                0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }

  const bool add_bias = ep.bias != nullptr && blockIdx.z == 0;
  if (!ep.c_f32) {
    // ---- LDS-staged bf16 epilogue (32-row halves of the wave tile)
    constexpr int LDW = WCOLS + 8, CPR = WCOLS / 8, NCH = 32 * CPR / 64;
    static_assert(32 * LDW * 2 * W <= STAGES * STAGE, "epilogue slab");
    static_assert(NCH >= 1 && (32 * CPR) % 64 == 0, "epilogue lanes");
    bf16_t* slab = (bf16_t*)(smem + wid * (32 * LDW * 2));
    float bv[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * WCOLS + 16 * j + (lane & 15);
      bv[j] = (add_bias && col < a.N) ? bf2f(ep.bias[col]) : 0.f;
    }
    cd_barrier();
    const int cbase = n0 + wn * WCOLS;
#pragma unroll
    for (int h = 0; h < (TM + 1) / 2; ++h) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = 2 * h + ii;
        if (i >= TM) break;
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[i][j][r] * ep.alpha + bv[j];
            if (ep.relu) v = fmaxf(v, 0.f);
            slab[(16 * ii + 4 * (lane >> 4) + r) * LDW + 16 * j + (lane & 15)] = f2bf(v);
          }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int hrows = min(32, WROWS - 32 * h);
#pragma unroll
      for (int u = 0; u < NCH; ++u) {
        const int idx = u * 64 + lane, lr = idx / CPR, ch = idx % CPR;
        const int row = m0 + wm * WROWS + 32 * h + lr;
        const int col = cbase + ch * 8;
        if (lr >= hrows || row >= a.M || col >= a.N) continue;
        bf16_t* dst = (bf16_t*)ep.c + (long)row * ep.ldc + col;
        const bf16_t* src = slab + lr * LDW + ch * 8;
        if (col + 8 <= a.N) {
          uint4 v = *(const uint4*)src;
          uint32_t* vw = (uint32_t*)&v;
          if (ep.mask) {
            const uint4 mk = *(const uint4*)(ep.mask + (long)row * ep.ldm + col);
            const uint32_t* mw = (const uint32_t*)&mk;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const uint32_t m2 = mw[e];
              const bool lo = (m2 & 0x8000u) == 0 && (m2 & 0x7fffu) != 0;
              const bool hi = (m2 & 0x80000000u) == 0 && (m2 & 0x7fff0000u) != 0;
              vw[e] &= (lo ? 0x0000ffffu : 0u) | (hi ? 0xffff0000u : 0u);
            }
          }
          if (ep.mode == 1) {
            const uint4 o = *(const uint4*)dst;
            const uint32_t* ow = (const uint32_t*)&o;
#pragma unroll
            for (int e = 0; e < 4; ++e)
              vw[e] = pack_bf2(bf2f((bf16_t)(vw[e] & 0xffff)) + bf2f((bf16_t)(ow[e] & 0xffff)),
                               bf2f((bf16_t)(vw[e] >> 16)) + bf2f((bf16_t)(ow[e] >> 16)));
          }
          *(uint4*)dst = v;
        } else {
          for (int e = 0; e < 8 && col + e < a.N; ++e) {
            float v = bf2f(src[e]);
            if (ep.mask && bf2f(ep.mask[(long)row * ep.ldm + col + e]) <= 0.f) v = 0.f;
            if (ep.mode == 1) v += bf2f(dst[e]);
            dst[e] = f2bf(v);
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    return;
  }

  // ---- fp32 output in the MFMA C layout: col = lane&15, row = (lane>>4)*4 + r
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WCOLS + 16 * j + (lane & 15);
    if (col >= a.N) continue;
    const float bv = add_bias ? bf2f(ep.bias[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * WROWS + 16 * i + 4 * (lane >> 4) + r;
        if (row >= a.M) continue;
        float v = acc[i][j][r] * ep.alpha + bv;
        if (ep.relu) v = fmaxf(v, 0.f);
        if (ep.mask && bf2f(ep.mask[(long)row * ep.ldm + col]) <= 0.f) v = 0.f;
        float* c = (float*)ep.c + (long)row * ep.ldc + col;
        if (ep.mode == 2) atomicAdd(c, v);
        else if (ep.mode == 1) *c += v;
        else *c = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// host side: eligibility, tile choice, launch
// ---------------------------------------------------------------------------
inline bool gemm_dma_ok(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk,
                        int M, int N, int K, const Epi& ep) {
  if (K < 64 || K % 64 != 0 || M < 1 || N < 1) return false;
  if (lda % 8 || ldb % 8 || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return false;
  if (!ak && (M % 8 || M < 8)) return false;
  if (!bk && (N % 8 || N < 8)) return false;
  (void)ep;
  return true;
}

// cfg: 0 = 256x128 (8 waves, 3 stages, 144 KiB), 1 = 128x128 (4 waves, 3 stages,
// 96 KiB), 2 = 128x64 (2 waves, 3 stages, 72 KiB: 2 blocks/CU), 3 = 64x64
// (2 waves, 4 stages, 64 KiB: 2 blocks/CU). Every wave owns 64 rows.
struct GdChoice { int cfg; int splits; };

inline GdChoice gemm_dma_choose(int M, int N, int K, bool can_split) {
  static const int bm[4] = {256, 128, 128, 64}, bn[4] = {128, 128, 64, 64};
  int cfg = 3;
  for (int c = 0; c < 4; ++c) {
    const long tiles = (long)cdiv(M, bm[c]) * cdiv(N, bn[c]);
    if (M <= bm[c] / 2 && c < 3) continue;            // mostly-empty row tiles
    if (tiles >= 256) { cfg = c; break; }
  }
  GdChoice ch{cfg, 1};
  const long tiles = (long)cdiv(M, bm[cfg]) * cdiv(N, bn[cfg]);
  const int ktiles = K / 64;
  if (can_split && tiles < 128 && ktiles >= 8) {
    int sp = (int)((256 + tiles - 1) / tiles);
    if (sp > ktiles / 4) sp = ktiles / 4;
    ch.splits = sp < 1 ? 1 : sp;
  }
  return ch;
}

template <int BM, int BN, int WM, int WN, int ST>
inline void gd_launch(const GDArgs& g, const Epi& ep, bool ak, bool bk, int z, hipStream_t s) {
  const dim3 grid(cdiv(g.M, BM) * cdiv(g.N, BN), 1, z), blk(64 * WM * WN);
  if (ak && bk) hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, WM, WN, true, true, ST>), grid, blk, 0, s, g, ep);
  else if (ak) hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, WM, WN, true, false, ST>), grid, blk, 0, s, g, ep);
  else if (bk) hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, WM, WN, false, true, ST>), grid, blk, 0, s, g, ep);
  else hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, WM, WN, false, false, ST>), grid, blk, 0, s, g, ep);
}

inline void launch_gemm_dma(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk,
                            int M, int N, int K, const Epi& ep, int cfg, int splits, hipStream_t s) {
  const int ktiles = K / 64;
  int kps = cdiv(ktiles, splits < 1 ? 1 : splits);
  const int z = cdiv(ktiles, kps);
  GDArgs g{A, lda, B, ldb, M, N, K, kps};
  switch (cfg) {
    case 0: gd_launch<256, 128, 4, 2, 3>(g, ep, ak, bk, z, s); break;
    case 1: gd_launch<128, 128, 2, 2, 3>(g, ep, ak, bk, z, s); break;
    case 2: gd_launch<128, 64, 2, 1, 3>(g, ep, ak, bk, z, s); break;
    default: gd_launch<64, 64, 1, 2, 4>(g, ep, ak, bk, z, s); break;
  }
}

}  // namespace tam
