// tiresias_amd — LDS-DMA MFMA GEMM for every operand majority, three tile
// shapes: 256x256 (8 waves, big GEMMs), 128x128 (4 waves, two blocks per
// CU, the mid-size GEMMs of the zoo: FFN / LSTM-gate projections and their
// gradients) and 64x128 (4 waves of 32x64, K-major A: the N = 512
// projections, 256 tiles = one per CU). C[M][N] (+)= A . B, bf16 in, fp32
// accumulate.
//
//   A: K-major [M][K] (AK) or M-major [K][M];  B: K-major [N][K] (BK) or N-major [K][N]
//
// MI355X-first structure (cdna_hip_programming.md §5 "The 256^2 8-phase
// template", T1-T5, T10):
//  * 256^2: 512 threads = 8 waves as 2 (M) x 4 (N), 128x64 outputs per wave
//    (8x4 tiles of v_mfma_f32_16x16x32_bf16, 128 fp32 accumulators / lane);
//    128^2: 256 threads = 4 waves as 2 x 2, 64x64 per wave.
//  * Both operands are staged HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4,
//    no VGPR round trip). Each operand tile is split in two half-tiles by the
//    C-quadrant that reads it (A: the wave's upper / lower 64 rows, B: its
//    left / right 32 columns); per K-tile a wave runs 4 phases = 4 quadrants
//    of 16 MFMAs, fragments held in registers between phases.
//  * K-major half-tile image: [128 rows][64 k] (128-B rows), 16-B chunk c of
//    row r stored at c ^ ((r>>1)&7): ds_read_b128 fragment reads conflict-free.
//    MN-major half-tile image: [64 k][128 cols] (256-B rows), 8-B chunk c of
//    row r at c ^ swz(r) (multiples of 4, so 16-B DMA granules stay whole),
//    read with the ds_read_b64_tr_b16 hardware transpose (T10). In both the
//    swizzle is applied to the per-lane SOURCE address (LDS-DMA writes
//    lane-linear; guide rule 21).
//  * Two LDS stages (2 x 64 KiB). Each half-tile (2 DMA per thread) is
//    refilled as EARLY as its buffer allows (>= 2 phases after its last
//    reader), so every DMA has >= 3 phases of MFMA work to land:
//        phase:   p1        p2     p3        p4
//        reads:   AL, BL    BH     AH        -
//        refill:  AH(t+1)   -      AL(t+2)   BL(t+2), BH(t+2)
//    and ONE counted `s_waitcnt vmcnt(6)` per K-tile (in p4, before its
//    first barrier) retires tile t+1 while tile t+2's three half-tiles stay
//    in flight: the DMA pipeline never drains inside the loop.
//  * One raw s_barrier per phase (after its MFMA cluster), MFMA clusters
//    bracketed by s_setprio (T5); fragment reads wait per fragment, so a
//    cluster's first MFMAs start while its later reads are in flight.
//  * XCD-aware bijective block remap + grouped-M tile order (T1); split-K
//    over blockIdx.z (fp32 atomic epilogue) when the tile grid underfills
//    the 256 CUs.
#pragma once
#include "tam/igemm.h"

namespace tam {

constexpr int P8_BK = 64;

typedef __attribute__((address_space(3))) void p8_lds_t;

struct P8Args {
  const bf16_t* A;
  long lda;
  const bf16_t* B;
  long ldb;
  int M, N, K;
  int kps;   // K-tiles per split (blockIdx.z)
  int group = 4;   // M-tiles per tile-order group (L2 reuse of B panels)
};

// Tile geometry: BM x BN block, 2 (M) x WNW (N) waves.
template <int BM, int BN, int WNW>
struct P8Geo {
  static constexpr int NW = 2 * WNW, THREADS = 64 * NW;
  static constexpr int WTM = BM / 2, WTN = BN / WNW;       // wave tile
  static constexpr int QM = WTM / 2, QN = WTN / 2;         // quadrant (one phase)
  static constexpr int FI = QM / 16, FJ = QN / 16;         // MFMA tiles per quadrant
  static constexpr int AROWS = BM / 2, BCOLS = BN / 2;     // rows of an A / B half-tile
  static constexpr int AHALF = AROWS * P8_BK * 2, BHALF = BCOLS * P8_BK * 2;
  static constexpr int STAGE = 2 * AHALF + 2 * BHALF;      // AL AH BL BH
  static constexpr int LDS = 2 * STAGE;
  // LDS-DMA instructions per thread per half-tile (16 B each): 2 for the
  // square tiles, 1 / 2 for the 64x128 tile's A / B halves
  static constexpr int DA = AHALF / (THREADS * 16), DB = BHALF / (THREADS * 16);
  static_assert(DA >= 1 && DB >= 1 && AHALF == THREADS * 16 * DA && BHALF == THREADS * 16 * DB,
                "whole DMA instructions per half");
  // DMAs left in flight by the per-K-tile counted wait: tile t+2's AL, BL, BH
  static constexpr int INFLIGHT = DA + 2 * DB;
};

// s_waitcnt vmcnt(N) with N a compile-time constant (inline asm needs a literal)
template <int N>
__device__ __forceinline__ void p8_vmcnt() {
  static_assert(N >= 0 && N <= 8, "p8_vmcnt: 0..8");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
}

// local row lr of a half-tile -> row / column offset in the block tile
//   A half h: rows wm*WTM + h*QM + (lr % QM), wm = lr / QM
//   B half h: cols wn*WTN + h*QN + (lr % QN), wn = lr / QN
template <int Q>
__device__ __forceinline__ int p8_row(int lr, int h) {
  return (lr / Q) * (2 * Q) + h * Q + (lr % Q);
}

// Issue one half-tile (D DMA instructions per thread). EXT = rows of the
// half-tile (K-major image) or its columns (MN-major image).
template <int Q, int EXT, int NW, bool KMAJ, int D = 2>
__device__ __forceinline__ void p8_issue(const bf16_t* __restrict__ base, long ld, int extent, int o0,
                                         int k0, char* half, int h, int wid, int lane) {
#pragma unroll
  for (int j = 0; j < D; ++j) {
    const int g = j * NW + wid;                // 1-KiB group of the half-tile
    if constexpr (KMAJ) {
      // 8 rows x 128 B per group; lane -> row 8g + lane/8, 16-B slot lane%8
      const int lr = g * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((lr >> 1) & 7);
      int r = o0 + p8_row<Q>(lr, h);
      r = r < extent ? r : extent - 1;         // rows past the edge are never stored
      const bf16_t* src = base + (long)r * ld + k0 + c * 8;
      __builtin_amdgcn_global_load_lds((const void*)src, (p8_lds_t*)(half + g * 1024), 16, 0, 0);
    } else {
      // [64 k][EXT cols] image; RPG k-rows x (EXT*2) B per group
      constexpr int GPR = EXT / 8, RPG = 64 / GPR;       // 16-B granules per row, rows per group
      const int kr = g * RPG + lane / GPR;
      const int gran = (lane % GPR) ^ (mnmaj_swz<EXT>(kr) >> 1);   // 8 columns per granule
      int col = o0 + p8_row<Q>(gran * 8, h);
      col = col + 8 <= extent ? col : extent - 8;                  // extent % 8 == 0
      const bf16_t* src = base + (long)(k0 + kr) * ld + col;
      __builtin_amdgcn_global_load_lds((const void*)src, (p8_lds_t*)(half + g * 1024), 16, 0, 0);
    }
  }
}

template <bool KMAJ, int EXT>
__device__ __forceinline__ s16x8_t p8_frag(const char* half, int lane, int lbase, int kk) {
  if constexpr (KMAJ) return read_frag_k(half, lane, lbase, kk);
  else return read_frag_mn<EXT>(half, lane, 32 * kk, lbase);
}

// raw s_barrier fenced for the COMPILER only (LDS reads / DMA issues stay on
// their side); emits no s_waitcnt, so DMAs stay in flight across it
__device__ __forceinline__ void p8_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// FINE: no blanket lgkmcnt(0) in front of the cluster -- the compiler's own
// per-fragment lgkmcnt waits let the first MFMAs start while later
// fragment reads are still in flight
template <int I0, int J0, bool FINE = false, int FI, int FJ, int TI, int TJ>
__device__ __forceinline__ void p8_mfma(f32x4_t (&acc)[TI][TJ], const s16x8_t (&fa)[FI][2],
                                        const s16x8_t (&fb)[FJ][2]) {
  if constexpr (!FINE) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j)
        acc[I0 + i][J0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(bf16x8_t, fa[i][kk]), __builtin_bit_cast(bf16x8_t, fb[j][kk]),
            acc[I0 + i][J0 + j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
  __builtin_amdgcn_sched_barrier(0);
}

// Output epilogue shared by the schedules: acc[TI][TJ] of a 2 x WNW wave
// grid, staged through the block's LDS (smem, >= NW * 32 * (WTN + 4) * 4 B).
// J0 / NJ: only fragment columns [J0, J0 + NJ) of every wave tile (the two K
// groups of gemm8p_ks2_kernel store one half each)
template <int BM, int BN, int WNW, int TI, int TJ, int J0 = 0, int NJ = TJ>
__device__ __forceinline__ void p8_epilogue(const P8Args& a, const Epi& ep, f32x4_t (&acc)[TI][TJ], char* smem,
                                            const int m0, const int n0, const int kz, const int wid,
                                            const int lane) {
  using G = P8Geo<BM, BN, WNW>;
  const int wm = wid / WNW, wn = wid % WNW;

  const bool add_bias = ep.bias != nullptr && kz == 0;
  static_assert(J0 >= 0 && NJ >= 1 && J0 + NJ <= TJ, "fragment column range");
  const int rbase = m0 + wm * G::WTM, cbase = n0 + wn * G::WTN + 16 * J0;
  constexpr int WTN = 16 * NJ;   // columns this epilogue stores per wave
  float bv[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    if (j < J0 || j >= J0 + NJ) continue;
    const int col = cbase + 16 * (j - J0) + (lane & 15);
    bv[j] = (add_bias && col < a.N) ? bf2f(ep.bias[col]) : 0.f;
  }
  // ---- bf16 output, plain store / accumulate (+ relu-backward mask read in
  // the same 16-B units): LDS-staged, 16-B row chunks
  const bool mask16 = ep.mask == nullptr || ((ep.ldm & 7) == 0 && (((uintptr_t)ep.mask) & 15) == 0);
  if (!ep.c_f32 && mask16 && (ep.ldc & 7) == 0 && (((uintptr_t)ep.c) & 15) == 0) {
    constexpr int LDW = WTN + 8, CPR = WTN / 8;
    bf16_t* slab = (bf16_t*)(smem + wid * (32 * LDW * 2));
#pragma unroll
    for (int h = 0; h < TI / 2; ++h) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = J0; j < J0 + NJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[2 * h + ii][j][r] * ep.alpha + bv[j];
            if (ep.relu) v = fmaxf(v, 0.f);
            slab[(16 * ii + 4 * (lane >> 4) + r) * LDW + 16 * (j - J0) + (lane & 15)] = f2bf(v);
          }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < 32 * CPR / 64; ++u) {
        const int idx = u * 64 + lane, lr = idx / CPR, ch = idx % CPR;
        const int row = rbase + 32 * h + lr, col = cbase + ch * 8;
        if (row >= a.M || col >= a.N) continue;
        bf16_t* dst = (bf16_t*)ep.c + (long)row * ep.ldc + col;
        const bf16_t* src = slab + lr * LDW + ch * 8;
        if (col + 8 <= a.N) {
          uint4 v = *(const uint4*)src;
          if (ep.mask) {
            // zero where the mask (a ReLU output) is <= 0: bf16 sign clear and
            // magnitude non-zero <=> > 0
            const uint4 mk = *(const uint4*)(ep.mask + (long)row * ep.ldm + col);
            const uint32_t* mw = (const uint32_t*)&mk;
            uint32_t* vw = (uint32_t*)&v;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const uint32_t m2 = mw[e];
              const bool lo = (m2 & 0x8000u) == 0 && (m2 & 0x7fffu) != 0;
              const bool hi = (m2 & 0x80000000u) == 0 && (m2 & 0x7fff0000u) != 0;
              vw[e] &= (lo ? 0x0000ffffu : 0u) | (hi ? 0xffff0000u : 0u);
            }
          }
          if (ep.mode == 1) {
            uint32_t* vw = (uint32_t*)&v;
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
  // ---- fp32 output, store / accumulate / split-K slab: LDS-staged, 16-B row chunks
  if (ep.c_f32 && ep.mode != 2 && !ep.mask && (ep.ldc & 3) == 0 && (((uintptr_t)ep.c) & 15) == 0 &&
      (ep.mode != 3 || (ep.zstride & 3) == 0)) {
    constexpr int LDF = WTN + 4, CPR = WTN / 4;
    float* slab = (float*)(smem + wid * (32 * LDF * 4));
    float* cz = (float*)ep.c + (ep.mode == 3 ? kz * ep.zstride : 0);
#pragma unroll
    for (int h = 0; h < TI / 2; ++h) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = J0; j < J0 + NJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[2 * h + ii][j][r] * ep.alpha + bv[j];
            if (ep.relu) v = fmaxf(v, 0.f);
            slab[(16 * ii + 4 * (lane >> 4) + r) * LDF + 16 * (j - J0) + (lane & 15)] = v;
          }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < 32 * CPR / 64; ++u) {
        const int idx = u * 64 + lane, lr = idx / CPR, ch = idx % CPR;
        const int row = rbase + 32 * h + lr, col = cbase + ch * 4;
        if (row >= a.M || col >= a.N) continue;
        float* dst = cz + (long)row * ep.ldc + col;
        const float* src = slab + lr * LDF + ch * 4;
        if (col + 4 <= a.N) {
          float4 v = *(const float4*)src;
          if (ep.mode == 1) {
            const float4 o = *(const float4*)dst;
            v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
          }
          *(float4*)dst = v;
        } else {
          for (int e = 0; e < 4 && col + e < a.N; ++e) dst[e] = ep.mode == 1 ? dst[e] + src[e] : src[e];
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    return;
  }
  // ---- general epilogue (atomics / relu-mask): C/D map of 16x16x32:
  // col = lane&15, row = (lane>>4)*4 + r
#pragma unroll
  for (int j = J0; j < J0 + NJ; ++j) {
    const int col = cbase + 16 * (j - J0) + (lane & 15);
    if (col >= a.N) continue;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + 16 * i + 4 * (lane >> 4) + r;
        if (row >= a.M) continue;
        float v = acc[i][j][r] * ep.alpha + bv[j];
        if (ep.relu) v = fmaxf(v, 0.f);
        if (ep.mask && bf2f(ep.mask[(long)row * ep.ldm + col]) <= 0.f) v = 0.f;
        const long off = (long)row * ep.ldc + col;
        if (ep.c_f32) {
          float* c = (float*)ep.c;
          if (ep.mode == 3) c[off + kz * ep.zstride] = v;
          else if (ep.mode == 2) atomicAdd(c + off, v);
          else if (ep.mode == 1) c[off] += v;
          else c[off] = v;
        } else {
          bf16_t* c = (bf16_t*)ep.c;
          if (ep.mode == 1) v += bf2f(c[off]);
          c[off] = f2bf(v);
        }
      }
    }
  }
}

// One schedule (measured best of six in round 2, profiles/r2/gemm8p_sched_ab.json;
// the other five were deleted in round 5): one barrier per phase, B fragments
// read before A (pinned order), and per-fragment lgkmcnt waits instead of a
// blanket lgkmcnt(0) in front of each MFMA cluster.
// The kernel body over one tile: bid = the (XCD-remapped) tile index within
// the M x N tile grid, kz = the K-split slice. Shared by gemm8p_kernel and the
// grouped launch (gemm8p_grouped_kernel: many independent problems, one grid).
// tile index -> (m0, n0): grouped-M order (a.group M-tiles per group) so
// consecutive tiles share B panels in L2
template <int BM, int BN>
__device__ __forceinline__ void p8_tile_origin(const P8Args& a, const int bid, int& m0, int& n0) {
  const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
  const int GROUP = a.group;
  const int per_group = GROUP * tiles_n;
  const int grp = bid / per_group;
  const int first_m = grp * GROUP;
  const int gsize = min(tiles_m - first_m, GROUP);
  m0 = (first_m + (bid % per_group) % gsize) * BM;
  n0 = ((bid % per_group) / gsize) * BN;
}

// kt_lo / kt_hi >= 0: an explicit K-tile range (stream-K segments); else
// slice kz of a.kps K-tiles
// KS > 1: KS groups of the tile's waves in one block, group g running the
// g-th of KS equal parts of the block's K range on an LDS image of its own
// (the caller guarantees an even split: every group meets the same barriers),
// then the partial tiles summed through LDS and stored by group 0. For tile
// grids of one block per CU (the N = 512 projections) it puts two waves on
// every SIMD without a split-K slab pass.
template <int BM, int BN, int WNW, bool AK, bool BK, int KS = 1>
__device__ __forceinline__ void gemm8p_body(const P8Args& a, const Epi& ep, const int bid, const int kz,
                                            const int kt_lo = -1, const int kt_hi = -1) {
  using G = P8Geo<BM, BN, WNW>;
  constexpr bool FINE = true;
  constexpr int FI = G::FI, FJ = G::FJ, TI = 2 * FI, TJ = 2 * FJ;
  __shared__ __attribute__((aligned(1024))) char smem_all[G::LDS * KS];
  const int grp = KS == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)threadIdx.x / G::THREADS);
  const int tid = KS == 1 ? (int)threadIdx.x : (int)threadIdx.x % G::THREADS, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WNW, wn = wid % WNW;
  char* smem = smem_all + grp * G::LDS;

  int m0, n0;
  p8_tile_origin<BM, BN>(a, bid, m0, n0);

  const int ktiles = a.K / P8_BK;
  int kt0 = kt_lo >= 0 ? kt_lo : kz * a.kps;
  int kt1 = kt_lo >= 0 ? kt_hi : min(ktiles, kt0 + a.kps);
  if constexpr (KS > 1) {
    const int part = (kt1 - kt0) / KS;
    kt0 += grp * part;
    kt1 = kt0 + part;
  }
  const int nk = kt1 - kt0;

  f32x4_t acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // stage s: [AL][AH][BL][BH]
  auto aptr = [&](int t, int h) { return smem + (t & 1) * G::STAGE + h * G::AHALF; };
  auto bptr = [&](int t, int h) { return smem + (t & 1) * G::STAGE + 2 * G::AHALF + h * G::BHALF; };
  auto issA = [&](int t, int h) {
    p8_issue<G::QM, G::AROWS, G::NW, AK, G::DA>(a.A, a.lda, a.M, m0, (kt0 + t) * P8_BK, aptr(t, h), h, wid, lane);
  };
  auto issB = [&](int t, int h) {
    p8_issue<G::QN, G::BCOLS, G::NW, BK, G::DB>(a.B, a.ldb, a.N, n0, (kt0 + t) * P8_BK, bptr(t, h), h, wid, lane);
  };

  if (nk > 0) {
    // prologue: tile 0 complete, tile 1's AL / BL / BH in flight
    issA(0, 0); issB(0, 0); issB(0, 1); issA(0, 1);
    if (nk > 1) {
      issA(1, 0); issB(1, 0); issB(1, 1);
      p8_vmcnt<G::INFLIGHT>();
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    p8_barrier();

    const int arow = wm * G::QM, bcol = wn * G::QN;   // local rows in the half images
    s16x8_t fa[FI][2], fb0[FJ][2], fb1[FJ][2];
    for (int t = 0; t < nk; ++t) {
      const char* AL = aptr(t, 0);
      const char* AH = aptr(t, 1);
      const char* BL = bptr(t, 0);
      const char* BH = bptr(t, 1);
      const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
      // ---- p1: quadrant (mh0, nh0); B fragments first (pinned
      // B-before-A issue order, guide §5 8-phase template)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < FJ; ++j) fb0[j][kk] = p8_frag<BK, G::BCOLS>(BL, lane, bcol + 16 * j, kk);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < FI; ++i) fa[i][kk] = p8_frag<AK, G::AROWS>(AL, lane, arow + 16 * i, kk);
      if (n1) issA(t + 1, 1);
      p8_mfma<0, 0, FINE>(acc, fa, fb0);
      p8_barrier();
      // ---- p2: quadrant (mh0, nh1)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < FJ; ++j) fb1[j][kk] = p8_frag<BK, G::BCOLS>(BH, lane, bcol + 16 * j, kk);
      p8_mfma<0, FJ, FINE>(acc, fa, fb1);
      p8_barrier();
      // ---- p3: quadrant (mh1, nh1)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < FI; ++i) fa[i][kk] = p8_frag<AK, G::AROWS>(AH, lane, arow + 16 * i, kk);
      if (n2) issA(t + 2, 0);
      p8_mfma<FI, FJ, FINE>(acc, fa, fb1);
      p8_barrier();
      // ---- p4: quadrant (mh1, nh0); retire tile t+1 (t+2's AL / BL / BH stay in flight)
      if (n2) {
        issB(t + 2, 0);
        issB(t + 2, 1);
        p8_vmcnt<G::INFLIGHT>();
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      p8_mfma<FI, 0, FINE>(acc, fa, fb0);
      p8_barrier();
    }
  }
  __syncthreads();   // LDS reuse by the epilogue
  if constexpr (KS > 1) {
    static_assert(KS == 2 && TJ % 2 == 0, "two K groups, two fragment-column halves");
    constexpr int JH = TJ / 2;
    static_assert(G::NW * TI * JH * 4 * 64 * 4 <= G::LDS, "half a partial tile fits a group's LDS");
    // group g keeps fragment columns [g JH, g JH + JH) of every wave tile: it
    // parks the other half of its partial tile in its own (now idle) LDS
    // image, lane-linear per (wave, fragment, element), adds the other
    // group's half of its own columns, and both groups store their halves
    float* mine = (float*)(smem_all + grp * G::LDS);
    const float* other = (const float*)(smem_all + (grp ^ 1) * G::LDS);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < JH; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          mine[(((wid * TI + i) * JH + j) * 4 + r) * 64 + lane] = grp == 0 ? acc[i][JH + j][r] : acc[i][j][r];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < JH; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float o = other[(((wid * TI + i) * JH + j) * 4 + r) * 64 + lane];
          if (grp == 0) acc[i][j][r] += o;
          else acc[i][JH + j][r] += o;
        }
    __syncthreads();   // partials read before the epilogue slabs reuse the images
    if (grp == 0) p8_epilogue<BM, BN, WNW, TI, TJ, 0, JH>(a, ep, acc, smem_all, m0, n0, kz, wid, lane);
    else p8_epilogue<BM, BN, WNW, TI, TJ, JH, JH>(a, ep, acc, smem_all + G::LDS, m0, n0, kz, wid, lane);
    return;
  }
  p8_epilogue<BM, BN, WNW>(a, ep, acc, smem_all, m0, n0, kz, wid, lane);
}

// the in-block two-group K split of gemm8p_body (KS = 2): 2 x the tile's waves
template <int BM, int BN, int WNW, bool AK, bool BK>
__global__ void __launch_bounds__(2 * 128 * WNW, 1) gemm8p_ks2_kernel(P8Args a, Epi ep) {
  gemm8p_body<BM, BN, WNW, AK, BK, 2>(a, ep, xcd_remap(blockIdx.x, gridDim.x), blockIdx.z);
}

template <int BM, int BN, int WNW, bool AK, bool BK>
void p8_launch_ks2(const P8Args& g, const Epi& ep, dim3 grid, hipStream_t s) {
  hipLaunchKernelGGL((gemm8p_ks2_kernel<BM, BN, WNW, AK, BK>), grid, dim3(2 * P8Geo<BM, BN, WNW>::THREADS), 0, s,
                     g, ep);
}

template <int BM, int BN, int WNW, bool AK, bool BK>
__global__ void __launch_bounds__(128 * WNW, (BM == 256 ? 1 : BM == 128 ? 2 : 3))
gemm8p_kernel(P8Args a, Epi ep) {
  gemm8p_body<BM, BN, WNW, AK, BK>(a, ep, xcd_remap(blockIdx.x, gridDim.x), blockIdx.z);
}

// One launcher per kernel variant. Each variant is explicitly instantiated
// in a translation unit of its own (csrc/kernels/gemm8p_*.hip): co-compiled
// instantiations of one kernel template share register-allocation context
// and perturb each other's code (cdna_hip_programming.md §5.4 rule 19).
template <int BM, int BN, int WNW, bool AK, bool BK>
void p8_launch_one(const P8Args& g, const Epi& ep, dim3 grid, hipStream_t s) {
  hipLaunchKernelGGL((gemm8p_kernel<BM, BN, WNW, AK, BK>), grid, dim3(P8Geo<BM, BN, WNW>::THREADS), 0, s,
                     g, ep);
}

#define TAM_P8_VARIANTS(X)                                                                     \
  X(256, 256, 4, true, true) X(256, 256, 4, true, false)                                       \
  X(256, 256, 4, false, true) X(256, 256, 4, false, false)                                     \
  X(128, 128, 2, true, true) X(128, 128, 2, true, false)                                       \
  X(128, 128, 2, false, true) X(128, 128, 2, false, false)                                     \
  X(64, 128, 2, true, true) X(64, 128, 2, true, false)
#define TAM_P8_EXTERN(BM, BN, W, AK, BK) \
  extern template void p8_launch_one<BM, BN, W, AK, BK>(const P8Args&, const Epi&, dim3, hipStream_t);
// the in-block K-split variants (tile code 65: 64 x 128, two K groups;
// 129: 128 x 128, two K groups)
#define TAM_P8_KS2_VARIANTS(X) \
  X(64, 128, 2, true, true) X(64, 128, 2, true, false) X(128, 128, 2, true, true) X(128, 128, 2, true, false)
#define TAM_P8_KS2_EXTERN(BM, BN, W, AK, BK) \
  extern template void p8_launch_ks2<BM, BN, W, AK, BK>(const P8Args&, const Epi&, dim3, hipStream_t);
#define TAM_P8_KS2_INST(BM, BN, W, AK, BK) \
  template void p8_launch_ks2<BM, BN, W, AK, BK>(const P8Args&, const Epi&, dim3, hipStream_t);
#define TAM_P8_INST(BM, BN, W, AK, BK) \
  template void p8_launch_one<BM, BN, W, AK, BK>(const P8Args&, const Epi&, dim3, hipStream_t);

// shape / layout conditions of the LDS-DMA kernels (tile >= 128)
inline bool gemm8p_ok(bool ak, bool bk, int M, int N, int K, long lda, long ldb) {
  if (K % P8_BK != 0 || K < P8_BK || M < 128 || N < 128) return false;
  if (lda % 8 != 0 || ldb % 8 != 0) return false;
  if (!ak && M % 8 != 0) return false;       // M-major A: 16-B column granules
  if (!bk && N % 8 != 0) return false;
  return true;
}

// tile: 256 (256x256, 8 waves), 128 (128x128, 4 waves) or 64 (64x128, 4
// waves of 32x64, K-major A only: the N = 512 projections of the
// Transformer, 4096 x 512 over 256 tiles = one per CU, ~3 blocks/CU of LDS)
inline bool gemm8p_tile_ok(int tile, bool ak) { return (tile != 64 && tile != 65 && tile != 129) || ak; }
void launch_gemm8p(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk, int M,
                   int N, int K, const Epi& ep, int splits, hipStream_t s, int tile = 256);
// split-K without atomics or a zeroing pass, any output dtype / epilogue:
// every K-slice writes its own fp32 slab of ws[splits][M][N], then one
// reduce pass sums the slabs and applies ep (bias / relu / mask / alpha /
// store or accumulate) — deterministic
void gemm8p_splitk(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk, int M,
                   int N, int K, const Epi& ep, int splits, float* ws, hipStream_t s, int tile = 256);
int gemm8p_slab_splits(int M, int N, int K, int tile = 256);
void gemm8p_slab_force(int sp);   // > 0: forced slab split count (A/B sweeps); 0: heuristic
// 128 or 256: the tile the auto policy picks for this shape
int gemm8p_tile(int M, int N, int K);
// stream-K schedule of the 256^2 kernel (gemm8p_sk.hip): one persistent
// block per CU over the flattened (tile, K-tile) space, fp32 partial tiles in
// ws (gemm8p_sk_ws_floats floats), one fixup pass applies ep
bool gemm8p_sk_ok(bool ak, bool bk, int M, int N, int K, long lda, long ldb);
long gemm8p_sk_ws_floats(int M, int N, int K);
void gemm8p_streamk(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk, int M, int N, int K,
                    const Epi& ep, float* ws, hipStream_t s);

}  // namespace tam
