// tiresias_amd — LDS-DMA implicit-GEMM convolution (fwd and stride-1 dgrad)
// for NHWC bf16 when the gathered operand has C % 64 == 0.
//
//   fwd  : Y[m=(n,p,q)][k]  = sum_{r,s,c} X[n, p*st-pad+r, q*st-pad+s, c] W[k][r][s][c]
//   dgrad: dX[m=(n,h,w)][c] = sum_{r,s,k} dY[n, h+pad-r, w+pad-s, k] Wt[c][r][s][k]
//
// Why a second conv core (the register-staged igemm in igemm.h stays for odd
// shapes): a 128x128 tile at full MFMA rate needs ~39 TB/s of operand traffic
// (over the 34.5 TB/s L2), and its per-load div/mod gather is VALU work in the
// MFMA gaps. Here:
//   * BM = 256 output rows x BN (64/128/256) columns, BK = 64; waves 4 (M) x WN,
//     each wave a 64 x (BN/WN) block of 16x16x32 MFMAs;
//   * since C % 64 == 0 a whole K-tile is ONE filter tap (r,s) and 64 channels,
//     so the tap is wave-uniform (scalar bookkeeping per K-tile) and every row of
//     the tile is one contiguous 128-B segment: pixel base (precomputed once per
//     row per thread) + tap offset, or the 128-B zero row for padding taps;
//   * both operands go HBM/L2 -> LDS with global_load_lds_dwordx4 (lane-linear
//     1 KiB per wave instruction = 8 rows), the XOR bank swizzle applied on the
//     SOURCE chunk; fragment reads are the conflict-free read_frag_k;
//   * a 3-stage ring (BN <= 128; 2 stages at BN = 256) with one raw barrier per
//     K-tile: counted `s_waitcnt vmcnt` retires tile t (tile t+1 stays in
//     flight across the barrier), then tile t+2 is issued into the stage tile
//     t-1 used, then tile t is computed;
//   * XCD-aware bijective workgroup remap, grouped-M tile order.
#pragma once
#include <cstdlib>
#include "tam/igemm.h"
#include "tam/slab.h"

namespace tam {

typedef __attribute__((address_space(3))) void cd_lds_void_t;

// 256 B of zeros: the source of every padding tap / pixel-tail row (device
// globals are zero-initialised at load; never written)
static __device__ __attribute__((aligned(256))) bf16_t g_cd_zero[128];

// Every pass is expressed as taps over a row grid:
//   row m = (n, p, q) over P x Q; its base source pixel (p*stride + base_h,
//   q*stride + base_w); K-tile kt -> tap t = kt / (Cs/64), channel block
//   kt % (Cs/64); tap t reads source pixel base + (tap_dh[t], tap_dw[t]) and
//   B columns tap_kcol[t] + 64*block of the weight rows (row stride ldb).
//   fwd         : taps (r,s) -> (r, s), kcol (r*S+s)*C, base -pad
//   dgrad s=1   : taps (r,s) -> (pad-r, pad-s), kcol (r*S+s)*K over Wt, base 0
//   dgrad s>1   : one launch per output parity (ph,pw) over the parity
//                 sub-grid, taps r = ph+pad (mod s) -> ((ph+pad-r)/s, ...);
//                 the epilogue maps row (n,i,j) to pixel (n, i*s+ph, j*s+pw)
struct CDArgs {
  const bf16_t* src;   // gathered operand, NHWC [.][Hs][Ws][Cs]
  const bf16_t* wgt;   // B operand, K-major rows of stride ldb
  int M, Ng, Kd;       // GEMM dims (Kd = ntaps*Cs)
  int Hs, Ws, Cs;      // gather source geometry
  int P, Q;            // rows m = (n, p, q) over a P x Q grid
  int stride, base_h, base_w;
  long ldb;
  int ntaps;
  int tap_dh[9], tap_dw[9], tap_kcol[9];
  // output row map (omap != 0): row (n,p,q) -> pixel (n, p*osh+ooh, q*osw+oow) of oH x oW
  int omap, oH, oW, osh, osw, ooh, oow;
  // multiply-high dividers by Q, P and Cs / 64 (the row decode of the
  // prologue and the strided-dgrad epilogue, the tap of each K-tile): set by
  // the argument builders (cd_divs), never left at their defaults
  FastDiv fq, fp, fct;
};

inline void cd_divs(CDArgs& a) {
  a.fq = FastDiv(a.Q);
  a.fp = FastDiv(a.P);
  a.fct = FastDiv(a.Cs / 64 > 0 ? a.Cs / 64 : 1);
}

__device__ __forceinline__ long cd_out_row(const CDArgs& a, int m) {
  if (!a.omap) return m;
  const int t = a.fq.div(m), q = m - t * a.Q, n = a.fp.div(t), p = t - n * a.P;
  return ((long)n * a.oH + p * a.osh + a.ooh) * a.oW + q * a.osw + a.oow;
}

template <int N>
__device__ __forceinline__ void cd_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void cd_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Epilogue of the conv cores over one BM x BN accumulator tile (waves WM (M)
// x WN, each 4 x TN blocks of 16x16 MFMA outputs): bias / ReLU / ReLU-backward
// mask / accumulate, bf16 (LDS-staged 16-B row chunks) or fp32 stores, and the
// BatchNorm sums (Epi::stats, Epi::bnx) added into statistics shard `shard`.
// rmap(tile-local row) -> output row, or -1 for a row that is not stored;
// Ng = output columns; smem = the kernel's (free) staging LDS.
template <int BN, int WN, int BM, class RowMap>
__device__ __forceinline__ void cd_epilogue(f32x4_t (&acc)[4][BN / WN / 16], const Epi& ep, char* smem,
                                            const int n0, const int Ng, const int shard, RowMap rmap) {
  constexpr int WM = BM / 64;
  constexpr int W = WM * WN;
  constexpr int WCOLS = BN / WN;
  constexpr int TN = WCOLS / 16, TM = 4;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % WM, wn = wid / WM;
  const bool add_bias = ep.bias != nullptr;
  if (!ep.c_f32) {
    // ---- LDS-staged bf16 epilogue: each wave parks 32 rows of its tile in a
    // private padded LDS slab (the stage buffers are free after the barrier),
    // then writes whole 16-B row chunks (and reads the relu mask / the
    // accumulate operand in the same 16-B units) instead of 2-B scattered
    // stores from the MFMA C layout.
    constexpr int LDW = WCOLS + 8;                 // padded slab row (bf16)
    constexpr int CPR = WCOLS / 8, NCH = 32 * CPR / 64;
    static_assert(64 % CPR == 0, "a lane keeps one 8-channel chunk");
    bf16_t* slab = (bf16_t*)(smem + wid * (32 * LDW * 2));
    // BN statistics of the stored tile (ep.stats): each lane owns channel
    // chunk lane % CPR for every row it stores
    const bool stats = ep.stats != nullptr;
    const bool bnb = stats && ep.bnx != nullptr;   // BN-backward sums (see Epi::bnx)
    float ssum[8], ssq[8], bmu[8], brs[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) ssum[e] = ssq[e] = bmu[e] = brs[e] = 0.f;
    if (bnb) {
      // a lane keeps one 8-channel chunk for every row it stores
      const int c0 = n0 + wn * WCOLS + (lane % CPR) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) { bmu[e] = ep.bnmean[c0 + e]; brs[e] = ep.bnrstd[c0 + e]; }
    }
    float bv[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
      bv[j] = add_bias ? bf2f(ep.bias[n0 + wn * WCOLS + 16 * j + (lane & 15)]) : 0.f;
    cd_barrier();                                  // every wave is done with the stages
    const int cbase = n0 + wn * WCOLS;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = 2 * half + ii;
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
#pragma unroll
      for (int u = 0; u < NCH; ++u) {
        const int idx = u * 64 + lane, lr = idx / CPR, ch = idx % CPR;
        const long orow = rmap(wm * 64 + half * 32 + lr);
        if (orow >= 0) {
          uint4 v = *(const uint4*)(slab + lr * LDW + ch * 8);
          if (ep.mask) {
            const uint4 mk = *(const uint4*)(ep.mask + orow * ep.ldm + cbase + ch * 8);
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
          bf16_t* dst = (bf16_t*)ep.c + orow * ep.ldc + cbase + ch * 8;
          if (ep.mode == 1) {
            const uint4 o = *(const uint4*)dst;
            const uint32_t* ow = (const uint32_t*)&o;
            uint32_t* vw = (uint32_t*)&v;
#pragma unroll
            for (int e = 0; e < 4; ++e)
              vw[e] = pack_bf2(bf2f((bf16_t)(vw[e] & 0xffff)) + bf2f((bf16_t)(ow[e] & 0xffff)),
                               bf2f((bf16_t)(vw[e] >> 16)) + bf2f((bf16_t)(ow[e] >> 16)));
          }
          *(uint4*)dst = v;
          if (bnb) {
            const uint4 xv = *(const uint4*)(ep.bnx + orow * ep.ldc + cbase + ch * 8);
            const uint32_t* vw = (const uint32_t*)&v;
            const uint32_t* xw = (const uint32_t*)&xv;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float lo = bf2f((bf16_t)(vw[e] & 0xffff)), hi = bf2f((bf16_t)(vw[e] >> 16));
              const float xl = bf2f((bf16_t)(xw[e] & 0xffff)), xh = bf2f((bf16_t)(xw[e] >> 16));
              ssum[2 * e] += lo; ssq[2 * e] += lo * (xl - bmu[2 * e]) * brs[2 * e];
              ssum[2 * e + 1] += hi; ssq[2 * e + 1] += hi * (xh - bmu[2 * e + 1]) * brs[2 * e + 1];
            }
          } else if (stats) {
            const uint32_t* vw = (const uint32_t*)&v;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float lo = bf2f((bf16_t)(vw[e] & 0xffff)), hi = bf2f((bf16_t)(vw[e] >> 16));
              ssum[2 * e] += lo; ssq[2 * e] += lo * lo;
              ssum[2 * e + 1] += hi; ssq[2 * e + 1] += hi * hi;
            }
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (stats) {
      // lanes sharing a chunk -> the wave's 64 rows; then the WM waves of
      // one column slice in LDS (past the slabs), one fp64 atomic add per
      // channel per M-tile
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          ssum[e] += __shfl_xor(ssum[e], o, 64);
          ssq[e] += __shfl_xor(ssq[e], o, 64);
        }
      float* red = (float*)(smem + W * 32 * LDW * 2);      // [W][2 * WCOLS]
      if (lane < CPR) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          red[wid * 2 * WCOLS + lane * 8 + e] = ssum[e];
          red[wid * 2 * WCOLS + WCOLS + lane * 8 + e] = ssq[e];
        }
      }
      __syncthreads();
      if (wm == 0) {
        for (int e = lane; e < 2 * WCOLS; e += 64) {
          float t = 0.f;
#pragma unroll
          for (int k = 0; k < WM; ++k) t += red[(k + WM * wn) * 2 * WCOLS + e];
          unsafeAtomicAdd(ep.stats + (long)shard * 2 * Ng + (e < WCOLS ? cbase + e : Ng + cbase + (e - WCOLS)),
                          (double)t);
        }
      }
    }
    return;
  }

  // ---- fp32 output: C/D map of 16x16x32: col = lane&15, row = (lane>>4)*4 + r
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WCOLS + 16 * j + (lane & 15);
    if (col >= Ng) continue;
    const float bv = add_bias ? bf2f(ep.bias[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long orow = rmap(wm * 64 + 16 * i + 4 * (lane >> 4) + r);
        if (orow < 0) continue;
        float v = acc[i][j][r] * ep.alpha + bv;
        if (ep.relu) v = fmaxf(v, 0.f);
        if (ep.mask && bf2f(ep.mask[orow * ep.ldm + col]) <= 0.f) v = 0.f;
        float* c = (float*)ep.c + orow * ep.ldc + col;
        if (ep.mode == 1) *c += v;
        else *c = v;
      }
    }
  }
}

// one block's tile of one pass; bid = the block's (XCD-remapped) index within
// the pass's tile grid
// kt_hi >= 0: only K-tiles [kt_lo, kt_hi) (split-K slice); slab != null:
// the raw fp32 accumulators go to slab[m][Ng] (tile rows m, no row map, no
// epilogue) for cd_slab_reduce_kernel
template <int BN, int WN, int BM, int NST = 0>   // NST: LDS ring depth (0: 3 if it fits, else 2)
__device__ __forceinline__ void conv_dma_body(const CDArgs& a, const Epi& ep, const int bid, const int kt_lo = 0,
                                              const int kt_hi = -1, float* __restrict__ slab = nullptr) {
  constexpr int WM = BM / 64;             // waves along M (64 rows each)
  constexpr int W = WM * WN;              // waves
  constexpr int BK = 64;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int STAGES = NST ? NST : (3 * STAGE <= 160 * 1024 ? 3 : 2);
  constexpr int AG = BM / 8 / W;          // A 8-row groups per wave
  constexpr int BG = BN / 8 / W;          // B 8-row groups per wave
  constexpr int D = AG + BG;              // DMA instructions per thread per K-tile
  constexpr int WCOLS = BN / WN;          // columns per wave
  constexpr int TN = WCOLS / 16, TM = 4;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % WM, wn = wid / WM;

  const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.Ng + BN - 1) / BN;
  constexpr int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int grp = bid / per_group;
  const int first_m = grp * GROUP;
  const int gsize = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (bid % per_group) % gsize;
  const int tn = (bid % per_group) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-thread row state (rows fixed for the whole K loop)
  const int lrow = lane >> 3;
  int abase[AG], ah[AG], aw[AG];
#pragma unroll
  for (int j = 0; j < AG; ++j) {
    const int rr = (wid + W * j) * 8 + lrow;
    const int c = (lane & 7) ^ ((rr >> 1) & 7);
    const int m = m0 + rr;
    if (m < a.M) {
      const int t = a.fq.div(m), q = m - t * a.Q, n = a.fp.div(t), p = t - n * a.P;
      const int hb = p * a.stride + a.base_h;
      const int wb = q * a.stride + a.base_w;
      ah[j] = hb;
      aw[j] = wb;
      abase[j] = ((n * a.Hs + hb) * a.Ws + wb) * a.Cs + c * 8;
    } else {
      ah[j] = -(1 << 28);                  // every tap out of range -> zero row
      aw[j] = 0;
      abase[j] = c * 8;
    }
  }
  const bf16_t* bptr[BG];
#pragma unroll
  for (int j = 0; j < BG; ++j) {
    const int rr = (wid + W * j) * 8 + lrow;
    const int c = (lane & 7) ^ ((rr >> 1) & 7);
    int n = n0 + rr;
    n = n < a.Ng ? n : a.Ng - 1;           // clamp: columns past the edge are never stored
    bptr[j] = a.wgt + (long)n * a.ldb + c * 8;
  }
  const int ctiles = a.Cs / BK;
  const int nk = (kt_hi < 0 ? a.Kd / BK : kt_hi) - kt_lo;

  auto issue = [&](int t, int st) {
    char* sa = smem + st * STAGE;
    char* sb = sa + A_BYTES;
    const int kt = kt_lo + t;
    const int tp = a.fct.div(kt), ct = kt - tp * ctiles;
    const int dh = a.tap_dh[tp], dw = a.tap_dw[tp];
    const int toff = (dh * a.Ws + dw) * a.Cs + ct * BK;
    const int kcol = a.tap_kcol[tp] + ct * BK;
#pragma unroll
    for (int j = 0; j < AG; ++j) {
      const int h = ah[j] + dh, w = aw[j] + dw;
      const bool ok = (unsigned)h < (unsigned)a.Hs && (unsigned)w < (unsigned)a.Ws;
      const int rr = (wid + W * j) * 8 + lrow;
      const bf16_t* p = ok ? a.src + (abase[j] + toff)
                           : g_cd_zero + (((lane & 7) ^ ((rr >> 1) & 7)) * 8);
      __builtin_amdgcn_global_load_lds((const void*)p, (cd_lds_void_t*)(sa + (wid + W * j) * 1024),
                                       16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < BG; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(bptr[j] + kcol),
                                       (cd_lds_void_t*)(sb + (wid + W * j) * 1024), 16, 0, 0);
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
#pragma unroll
    for (int t = 0; t < STAGES - 1; ++t)
      if (t < nk) issue(t, t);
    for (int t = 0; t < nk; ++t) {
      // retire tile t; leave the (STAGES-2) younger tiles in flight
      if constexpr (STAGES == 3) {
        if (t + 1 < nk) cd_vm_wait<D>();
        else cd_vm_wait<0>();
      } else {
        cd_vm_wait<0>();
      }
      cd_barrier();
      if (t + STAGES - 1 < nk) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
      const int st = t % STAGES;
      const char* ta = smem + st * STAGE;
      const char* tb = ta + A_BYTES;
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        s16x8_t fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = read_frag_k(ta, lane, wm * 64 + 16 * i, kk);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = read_frag_k(tb, lane, wn * WCOLS + 16 * j, kk);
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

  if (slab) {
    // C/D map of 16x16x32: col = lane&15, row = (lane>>4)*4 + r
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * WCOLS + 16 * j + (lane & 15);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
          if (row < a.M) slab[(long)row * a.Ng + col] = acc[i][j][r];
        }
    }
    return;
  }
  cd_epilogue<BN, WN, BM>(acc, ep, smem, n0, a.Ng, tm % BN_SHARDS, [&](int lr) -> long {
    const int row = m0 + lr;
    return row < a.M ? cd_out_row(a, row) : -1L;
  });
}

// split-K over blockIdx.y: slice kz owns K-tiles [kz * kps, (kz+1) * kps) and
// writes its partial sums to ws[kz][M][Ng]
template <int BN, int WN, int BM = 256, int NST = 0>
__global__ void __launch_bounds__(BM / 64 * 64 * WN, NST == 2 ? 2 : 1) conv_dma_split_kernel(CDArgs a, float* ws,
                                                                                            int kps) {
  const int nk = a.Kd / 64;
  const int lo = blockIdx.y * kps;
  conv_dma_body<BN, WN, BM, NST>(a, Epi{}, xcd_remap(blockIdx.x, gridDim.x), lo, min(nk, lo + kps),
                                 ws + (long)blockIdx.y * a.M * a.Ng);
}

// C = epilogue(sum_z ws[z]) for the split conv: bf16 output rows through the
// pass's row map, bias / relu / relu-mask / accumulate, and the BatchNorm sums
// of the stored values (Epi::stats, sharded fp64 atomics) -- what cd_epilogue
// does for an unsplit tile. Block = (Ng/8 channel groups) x row lanes over a
// contiguous row range.
static __global__ void __launch_bounds__(256) cd_slab_reduce_kernel(const float* __restrict__ ws, int sp, CDArgs a,
                                                             Epi ep, int rows_per_block) {
  __shared__ float red[2 * 2048];
  const int vs = a.Ng / 8, rpp = 256 / vs;
  const int cg = threadIdx.x % vs, rl = threadIdx.x / vs;
  const int c = cg * 8;
  float ssum[8], ssq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) ssum[e] = ssq[e] = 0.f;
  const long plane = (long)a.M * a.Ng;
  if (rl < rpp) {
    float bv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = ep.bias ? bf2f(ep.bias[c + e]) : 0.f;
    const int r0 = blockIdx.x * rows_per_block, r1 = min(a.M, r0 + rows_per_block);
    for (int m = r0 + rl; m < r1; m += rpp) {
      const float* src = ws + (long)m * a.Ng + c;
      float4 lo = *(const float4*)src, hi = *(const float4*)(src + 4);
      for (int z = 1; z < sp; ++z) {
        const float4 l2 = *(const float4*)(src + z * plane), h2 = *(const float4*)(src + z * plane + 4);
        lo.x += l2.x; lo.y += l2.y; lo.z += l2.z; lo.w += l2.w;
        hi.x += h2.x; hi.y += h2.y; hi.z += h2.z; hi.w += h2.w;
      }
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      const long orow = cd_out_row(a, m);
      bf16_t* dst = (bf16_t*)ep.c + orow * ep.ldc + c;
      uint4 mk = make_uint4(0u, 0u, 0u, 0u), old = make_uint4(0u, 0u, 0u, 0u);
      if (ep.mask) mk = *(const uint4*)(ep.mask + orow * ep.ldm + c);
      if (ep.mode == 1) old = *(const uint4*)dst;
      const uint32_t* mw = (const uint32_t*)&mk;
      const uint32_t* ow = (const uint32_t*)&old;
      uint32_t out[4];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = v[e] * ep.alpha + bv[e];
        if (ep.relu) t = fmaxf(t, 0.f);
        if (ep.mask) {
          const uint32_t mb = (mw[e >> 1] >> (16 * (e & 1))) & 0xffffu;
          if ((mb & 0x8000u) || !(mb & 0x7fffu)) t = 0.f;     // mask <= 0
        }
        if (ep.mode == 1) t = bf2f(f2bf(t)) + bf2f((bf16_t)((ow[e >> 1] >> (16 * (e & 1))) & 0xffffu));
        v[e] = bf2f(f2bf(t));                                 // the stored value
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) out[e] = pack_bf2(v[2 * e], v[2 * e + 1]);
      *(uint4*)dst = make_uint4(out[0], out[1], out[2], out[3]);
      if (ep.stats) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { ssum[e] += v[e]; ssq[e] += v[e] * v[e]; }
      }
    }
  }
  if (!ep.stats) return;
  // row lanes of one channel group -> LDS (float atomics) -> one fp64
  // atomic per channel per block into shard blockIdx % BN_SHARDS
  for (int e = threadIdx.x; e < 2 * a.Ng; e += 256) red[e] = 0.f;
  __syncthreads();
  if (rl < rpp) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      atomicAdd(&red[c + e], ssum[e]);
      atomicAdd(&red[a.Ng + c + e], ssq[e]);
    }
  }
  __syncthreads();
  double* sh = ep.stats + (long)(blockIdx.x % BN_SHARDS) * 2 * a.Ng;
  for (int e = threadIdx.x; e < 2 * a.Ng; e += 256) unsafeAtomicAdd(sh + e, (double)red[e]);
}

// NST = 2 on the 128-row tile (a 64 KiB ring, two blocks per CU) measured
// ResNet-50 9.72 -> 9.76 ms (profiles/r4/conv128_nst2_ab.log): not launched
template <int BN, int WN, int BM = 256, int NST = 0>
__global__ void __launch_bounds__(BM / 64 * 64 * WN, NST == 2 ? 2 : 1) conv_dma_kernel(CDArgs a, Epi ep) {
  conv_dma_body<BN, WN, BM, NST>(a, ep, xcd_remap(blockIdx.x, gridDim.x));
}

// Several independent passes sharing one epilogue in ONE launch: the parity
// classes of a strided dgrad (each a stride-1 sub-convolution over a quarter
// of the dX pixels, 1-4 taps). Launched separately each class is a grid of
// tens of blocks on 256 CUs (ResNet-50's 7x7 / 14x14 stages); together they
// fill the chip. Pass c owns blocks [t0[c], t0[c+1]) after the XCD remap.
constexpr int CD_MULTI = 4;
struct CDMulti {
  CDArgs a[CD_MULTI];
  int t0[CD_MULTI + 1];
  int n;
};

template <int BN, int WN, int BM = 256>
__global__ void __launch_bounds__(BM / 64 * 64 * WN, 1) conv_dma_multi_kernel(CDMulti m, Epi ep) {
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  int c = 0;
  while (c + 1 < m.n && bid >= m.t0[c + 1]) ++c;
  conv_dma_body<BN, WN, BM>(m.a[c], ep, bid - m.t0[c]);
}

// ===========================================================================
// Halo-tile conv for 64-channel 3x3 stride-1 passes (fwd over X, stride-1
// dgrad over dY): ResNet-50's 56x56 stage, VGG-16's 224x224 / 112x112 layers.
//
// The LDS-DMA core above gathers A per tap, so a 3x3 pass with C = 64 reads
// its source 9 times through L2 (measured ~5-6 TB/s of tap re-reads: the
// pass is bound by them, 57-300 TF/s). Here a block owns a 4 x 56 output
// tile (224 rows of the GEMM, 4 waves of 64 rows, 32 masked) and 64 output
// channels; its source PATCH -- 6 x 58 pixels x 64 channels incl. the halo
// and zero padding -- is staged ONCE by LDS-DMA (44 KiB, XOR-swizzled by
// patch pixel as the K-major tile image), and every tap's A fragment is read
// from the patch at a per-lane shifted pixel. B (64 x 64 weights of a tap,
// 8 KiB) streams through a 3-slot ring, tap t+2 issued while tap t computes.
// 68 KiB of LDS: two blocks per CU, one's patch load under the other's MFMAs.
// The epilogue is the conv cores' (bias / ReLU / mask / BN sums).
// ===========================================================================
constexpr int CH_TR = 4, CH_TQ = 56;                 // output tile
constexpr int CH_PR = CH_TR + 2, CH_PW = CH_TQ + 2;  // source patch
constexpr int CH_NP = CH_PR * CH_PW;                 // 348 pixels
constexpr int CH_GROUPS = (CH_NP + 7) / 8;           // 1-KiB DMA groups (44)
constexpr int CH_PATCH = CH_GROUPS * 1024;
constexpr int CH_BSLOT = 64 * 64 * 2;

struct CHArgs {
  const bf16_t* src;   // [N][P][Q][64]
  const bf16_t* wgt;   // B rows [Ng][ldb]: a tap's 64 k at column tap_kcol[t]
  long ldb;
  int N, P, Q, Ng;     // output grid == source grid (3x3, stride 1, "same")
  int tap_oh[9], tap_ow[9], tap_kcol[9];   // patch offsets in [0, 2]
};

static __global__ void __launch_bounds__(256, 2) conv_halo_kernel(CHArgs a, Epi ep) {
  __shared__ __attribute__((aligned(1024))) char smem[CH_PATCH + 3 * CH_BSLOT];
  char* sp = smem;
  char* sb = smem + CH_PATCH;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // tile (n, p0, q0) x column block tn; tn innermost so both column blocks
  // of a patch run together (the second patch read hits L2)
  const int tiles_n = a.Ng / 64, tq = a.Q / CH_TQ, tp = a.P / CH_TR;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = bid % tiles_n;
  const int sidx = bid / tiles_n;                 // spatial tile
  const int q0 = (sidx % tq) * CH_TQ;
  const int p0 = ((sidx / tq) % tp) * CH_TR;
  const int n = sidx / (tq * tp);
  const int n0 = tn * 64;

  // ---- patch: group g = wid + 4j holds patch pixels 8g .. 8g+7
#pragma unroll
  for (int j = 0; j < (CH_GROUPS + 3) / 4; ++j) {
    const int g = wid + 4 * j;
    if (g < CH_GROUPS) {
      const int i = 8 * g + (lane >> 3);
      const int pr = i / CH_PW, pc = i % CH_PW;
      const int h = p0 - 1 + pr, w = q0 - 1 + pc;
      const int c = (lane & 7) ^ ((i >> 1) & 7);
      const bool ok = i < CH_NP && (unsigned)h < (unsigned)a.P && (unsigned)w < (unsigned)a.Q;
      const bf16_t* src = ok ? a.src + (((long)n * a.P + h) * a.Q + w) * 64 + c * 8 : g_cd_zero + c * 8;
      __builtin_amdgcn_global_load_lds((const void*)src, (cd_lds_void_t*)(sp + g * 1024), 16, 0, 0);
    }
  }
  // ---- B ring: tap t -> slot t % 3; rows rr = (wid + 4j)*8 + lane/8
  const bf16_t* brow[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int rr = (wid + 4 * j) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((rr >> 1) & 7);
    brow[j] = a.wgt + (long)(n0 + rr) * a.ldb + c * 8;
  }
  auto issue_b = [&](int t) {
    char* dst = sb + (t % 3) * CH_BSLOT;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(brow[j] + a.tap_kcol[t]),
                                       (cd_lds_void_t*)(dst + (wid + 4 * j) * 1024), 16, 0, 0);
  };
  issue_b(0);
  issue_b(1);

  // ---- per-lane patch pixel of each A fragment row (center-less origin)
  int base[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int m = wid * 64 + 16 * i + (lane & 15);
    m = m < CH_TR * CH_TQ ? m : 0;                // masked rows: any valid pixel
    base[i] = (m / CH_TQ) * CH_PW + (m % CH_TQ);
  }
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int t = 0; t < 9; ++t) {
    // retire the patch and B(t); B(t+1) stays in flight
    if (t + 1 < 9) cd_vm_wait<2>();
    else cd_vm_wait<0>();
    cd_barrier();
    if (t + 2 < 9) issue_b(t + 2);                // slot (t+2)%3 was last read at tap t-1
    const char* tb = sb + (t % 3) * CH_BSLOT;
    const int toff = a.tap_oh[t] * CH_PW + a.tap_ow[t];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      s16x8_t fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[i] = *(const s16x8_t*)(sp + kmaj_off(base[i] + toff, 4 * kk + (lane >> 4)));
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = read_frag_k(tb, lane, 16 * j, kk);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8_t, fa[i]), __builtin_bit_cast(bf16x8_t, fb[j]), acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  const long rowbase = ((long)n * a.P + p0) * a.Q + q0;
  cd_epilogue<64, 1, 256>(acc, ep, smem, n0, a.Ng, sidx % BN_SHARDS, [&](int lr) -> long {
    if (lr >= CH_TR * CH_TQ) return -1L;
    return rowbase + (long)(lr / CH_TQ) * a.Q + (lr % CH_TQ);
  });
}

// 3x3 stride-1 "same" pass over a 64-channel source (fwd: CDArgs of
// cd_fwd_args; stride-1 dgrad: cd_dgrad_args) -> halo launch; false if the
// shape is not for this kernel
inline bool launch_conv_halo(const CDArgs& c, const Epi& ep, hipStream_t s) {
  if (c.Cs != 64 || c.ntaps != 9 || c.stride != 1 || c.omap || c.Ng % 64 != 0) return false;
  if (c.P != c.Hs || c.Q != c.Ws || c.P % CH_TR != 0 || c.Q % CH_TQ != 0) return false;
  const int N = c.M / (c.P * c.Q);
  if ((long)N * c.P * c.Q != c.M || (long)c.M * 64 >= (1L << 31) || (long)c.Ng * c.ldb >= (1L << 31))
    return false;
  CHArgs a{};
  a.src = c.src; a.wgt = c.wgt; a.ldb = c.ldb;
  a.N = N; a.P = c.P; a.Q = c.Q; a.Ng = c.Ng;
  for (int t = 0; t < 9; ++t) {
    a.tap_oh[t] = c.base_h + c.tap_dh[t] + 1;
    a.tap_ow[t] = c.base_w + c.tap_dw[t] + 1;
    a.tap_kcol[t] = c.tap_kcol[t];
    if (a.tap_oh[t] < 0 || a.tap_oh[t] > 2 || a.tap_ow[t] < 0 || a.tap_ow[t] > 2) return false;
  }
  const long blocks = (long)N * (c.P / CH_TR) * (c.Q / CH_TQ) * (c.Ng / 64);
  hipLaunchKernelGGL(conv_halo_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, ep);
  return true;
}

// Host-side eligibility + launch. Returns false when the shape is not for
// this core (caller falls back to the register-staged igemm).
// returns BN, or BN | 0x1000 for the 128-row tile variant.
// Cost model (fitted to profiles/conv_bench_r1_dma*.json): time ~ ceil(tiles /
// 256 CUs) x tile area / efficiency, efficiency 256x256 1.0, 256x128 0.92,
// 128x128 0.8. BN = 64 only for deep-K gathers (the 32 KiB A tile per 64
// columns is L2-bound at shallow K and loses to the igemm).
inline int conv_dma_pick_bn(int M, int Ng, int Kd, int force) {
  if (force == 2 && Ng % 128 == 0) return 128 | 0x1000;   // tests: the 128-row variant
  if (force) return Ng % 256 == 0 ? 256 : Ng % 128 == 0 ? 128 : Ng % 64 == 0 ? 64 : 0;
  const long tm = (M + 255) / 256, tm2 = (M + 127) / 128;
  double best = 1e30;
  int pick = 0;
  auto consider = [&](long tiles, double area, double eff, int code) {
    const double cost = (double)((tiles + 255) / 256) * area / eff;
    if (cost < best) { best = cost; pick = code; }
  };
  if (Ng % 256 == 0) consider(tm * (Ng / 256), 65536.0, 1.0, 256);
  if (Ng % 128 == 0) consider(tm * (Ng / 128), 32768.0, 0.92, 128);
  if (Ng % 128 == 0 && Kd >= 1024) consider(tm2 * (Ng / 128), 16384.0, 0.8, 128 | 0x1000);
  if (!pick && Ng % 64 == 0 && Kd >= 1024 && tm * (Ng / 64) >= 512) pick = 64;
  return pick;
}

// Split-K for a pass whose tile grid covers a fraction of the 256 CUs (the
// 7x7 / 14x14 stages of ResNet-50 at batch 64: 26-196 tiles). Every conv_dma
// tile runs one block per CU (the 3-stage rings are 96-192 KiB of LDS), so a
// launch costs ceil(blocks / CUs) block times; a split adds the fp32 slab
// round trip ((sp + 1) M Ng 4 B) and a reduce launch. Time model (us), per-CU
// rates as the pick model's efficiencies x ~2.4 TF/s (the measured 128-row
// 7x7 rate); returns the pick (tile code) and slices of the cheapest plan
// with >= 8 K-tiles per slice and <= 64 MiB of slabs.
struct CdSplit { int pick, sp; };
inline CdSplit cd_split_plan(const CDArgs& a, int pick0, int cus) {
  CdSplit best{pick0, 1};
  const int nk = a.Kd / 64;
  if (nk < 16) return best;
  double tbest = 1e30;
  const int codes[3] = {256, 128, 128 | 0x1000};
  const double eff[3] = {1.0, 0.92, 0.8};
  for (int c = 0; c < 3; ++c) {
    const int code = codes[c], bm = (code & 0x1000) ? 128 : 256, bn = code & 0xfff;
    if (a.Ng % bn) continue;
    if ((code & 0x1000) && a.Kd < 1024) continue;
    const long tiles = (long)((a.M + bm - 1) / bm) * (a.Ng / bn);
    const long slots = cus;
    for (int sp = 1; sp <= 8; ++sp) {
      if (sp > 1 && (nk / sp < 8 || (long)sp * a.M * a.Ng > (16L << 20))) break;
      const double block_us = 2.0 * bm * bn * (double)a.Kd / sp / (eff[c] * 2.4e6);
      const double waves = (double)((tiles * sp + slots - 1) / slots);
      double t = waves * block_us;
      if (sp > 1) t += (double)(sp + 1) * a.M * a.Ng * 4 / 4.0e6 + 3.0;
      if (t < tbest * 0.97) { tbest = t; best = CdSplit{code, sp}; }
    }
  }
  return best;
}

inline int cd_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      n = 256;
  }
  return n;
}

inline bool cd_base_ok(const CDArgs& a, int force) {
  // Kd >= 256: with fewer than 4 K-tiles the ring never fills (1x1 convs over
  // 64/128 channels measured slower than the igemm) — unless forced (tests,
  // strided-dgrad parity classes, where the igemm alternative is far worse)
  if (a.Cs % 64 != 0 || a.Kd % 64 != 0 || a.Kd < 64 || (a.Kd < 256 && !force)) return false;
  if (a.ntaps < 1 || a.ntaps > 9) return false;
  if ((long)a.Hs * a.Ws * a.Cs * ((a.M + a.P * a.Q - 1) / (a.P * a.Q)) >= (1L << 31)) return false;
  if ((long)a.Ng * a.ldb >= (1L << 31)) return false;
  return true;
}

// fp32 workspace (floats) a split launch of this pass would use; 0: unsplit
inline long conv_dma_split_ws(const CDArgs& a, int force = 0) {
  if (!cd_base_ok(a, force)) return 0;
  const int pick = conv_dma_pick_bn(a.M, a.Ng, a.Kd, force);
  if (!pick || force || (a.Ng / 8) > 256) return 0;
  const CdSplit p = cd_split_plan(a, pick, cd_cus());
  return p.sp > 1 ? (long)p.sp * a.M * a.Ng : 0;
}

// returns 0 (not for this core) or the tile height BM of the launch. ws /
// ws_floats: scratch for split-K (conv_dma_split_ws floats; none -> unsplit)
inline int launch_conv_dma(const CDArgs& a, const Epi& ep, hipStream_t s, int force = 0, float* ws = nullptr,
                           long ws_floats = 0) {
  if (!cd_base_ok(a, force)) return 0;
  const int pick = conv_dma_pick_bn(a.M, a.Ng, a.Kd, force);
  if (!pick) return 0;
  if (ws && !force && !ep.c_f32 && ep.mode != 2 && !ep.bnx && a.Ng / 8 <= 256) {
    const CdSplit p = cd_split_plan(a, pick, cd_cus());
    const int sp = p.sp;
    if (sp > 1 && (long)sp * a.M * a.Ng <= ws_floats) {
      const int nk = a.Kd / 64, kps = (nk + sp - 1) / sp, z = (nk + kps - 1) / kps;
      const bool t128 = (p.pick & 0x1000) != 0;
      const int bm = t128 ? 128 : 256, bn = p.pick & 0xfff;
      const dim3 grid((unsigned)(((a.M + bm - 1) / bm) * (a.Ng / bn)), (unsigned)z);
      if (t128) hipLaunchKernelGGL((conv_dma_split_kernel<128, 2, 128>), grid, dim3(256), 0, s, a, ws, kps);
      else if (bn == 256) hipLaunchKernelGGL((conv_dma_split_kernel<256, 2>), grid, dim3(512), 0, s, a, ws, kps);
      else if (bn == 128) hipLaunchKernelGGL((conv_dma_split_kernel<128, 2>), grid, dim3(512), 0, s, a, ws, kps);
      else hipLaunchKernelGGL((conv_dma_split_kernel<64, 1>), grid, dim3(256), 0, s, a, ws, kps);
      const int rpp = 256 / (a.Ng / 8);
      int rpb = (a.M + 511) / 512;                       // ~512 reducing blocks
      rpb = (rpb + rpp - 1) / rpp * rpp;
      if (rpb < rpp) rpb = rpp;
      hipLaunchKernelGGL(cd_slab_reduce_kernel, dim3((unsigned)((a.M + rpb - 1) / rpb)), dim3(256), 0, s, ws, z,
                         a, ep, rpb);
      return bm;
    }
  }
  if (pick & 0x1000) {
    const int tiles = ((a.M + 127) / 128) * (a.Ng / 128);
    hipLaunchKernelGGL((conv_dma_kernel<128, 2, 128>), dim3(tiles), dim3(256), 0, s, a, ep);
    return 128;
  }
  const int bn = pick;
  const int tiles = ((a.M + 255) / 256) * (a.Ng / bn);
  switch (bn) {
    case 256:
      hipLaunchKernelGGL((conv_dma_kernel<256, 2>), dim3(tiles), dim3(512), 0, s, a, ep);
      break;
    case 128:
      hipLaunchKernelGGL((conv_dma_kernel<128, 2>), dim3(tiles), dim3(512), 0, s, a, ep);
      break;
    default:
      hipLaunchKernelGGL((conv_dma_kernel<64, 1>), dim3(tiles), dim3(256), 0, s, a, ep);
      break;
  }
  return 256;
}

// One launch over the passes a[0..n) (same Ng, Cs % 64 == 0, 1 <= ntaps <= 9
// each; the caller checked them): tile by the cost model over the SUM of the
// passes' tiles. Returns false if no tile fits.
inline bool launch_conv_dma_multi(const CDArgs* a, int n, const Epi& ep, hipStream_t s) {
  if (n < 1 || n > CD_MULTI) return false;
  const int Ng = a[0].Ng;
  for (int i = 0; i < n; ++i)
    if (a[i].Ng != Ng || a[i].Cs % 64 || a[i].Kd % 64 || a[i].ntaps < 1 || a[i].ntaps > 9) return false;
  struct Cand { int bm, bn; double eff; };
  const Cand cands[3] = {{256, 256, 1.0}, {256, 128, 0.92}, {128, 128, 0.8}};
  int pick = -1;
  double best = 1e30;
  for (int k = 0; k < 3; ++k) {
    if (Ng % cands[k].bn) continue;
    long tiles = 0;
    for (int i = 0; i < n; ++i) tiles += (long)((a[i].M + cands[k].bm - 1) / cands[k].bm) * (Ng / cands[k].bn);
    const double cost = (double)((tiles + 255) / 256) * cands[k].bm * cands[k].bn / cands[k].eff;
    if (cost < best) { best = cost; pick = k; }
  }
  if (pick < 0) return false;
  CDMulti m{};
  m.n = n;
  int t = 0;
  for (int i = 0; i < n; ++i) {
    m.a[i] = a[i];
    m.t0[i] = t;
    t += ((a[i].M + cands[pick].bm - 1) / cands[pick].bm) * (Ng / cands[pick].bn);
  }
  m.t0[n] = t;
  for (int i = n + 1; i <= CD_MULTI; ++i) m.t0[i] = t;
  if (pick == 0)
    hipLaunchKernelGGL((conv_dma_multi_kernel<256, 2>), dim3(t), dim3(512), 0, s, m, ep);
  else if (pick == 1)
    hipLaunchKernelGGL((conv_dma_multi_kernel<128, 2>), dim3(t), dim3(512), 0, s, m, ep);
  else
    hipLaunchKernelGGL((conv_dma_multi_kernel<128, 2, 128>), dim3(t), dim3(256), 0, s, m, ep);
  return true;
}

// argument builders (host)
inline CDArgs cd_fwd_args(const bf16_t* x, const bf16_t* w, const ConvGeom& g) {
  CDArgs a{};
  a.src = x; a.wgt = w;
  a.M = g.N * g.P * g.Q; a.Ng = g.K; a.Kd = g.R * g.S * g.C;
  a.Hs = g.H; a.Ws = g.W; a.Cs = g.C; a.P = g.P; a.Q = g.Q;
  a.stride = g.stride; a.base_h = -g.pad; a.base_w = -g.pad;
  a.ldb = (long)g.R * g.S * g.C;
  a.ntaps = g.R * g.S;
  if (a.ntaps > 9) { a.ntaps = 0; cd_divs(a); return a; }
  for (int r = 0; r < g.R; ++r)
    for (int q = 0; q < g.S; ++q) {
      const int t = r * g.S + q;
      a.tap_dh[t] = r; a.tap_dw[t] = q; a.tap_kcol[t] = t * g.C;
    }
  cd_divs(a);
  return a;
}

// dgrad over Wt [C][R][S][K]; stride-s layers: parity class (ph, pw)
inline CDArgs cd_dgrad_args(const bf16_t* dy, const bf16_t* wt, const ConvGeom& g, int ph, int pw) {
  CDArgs a{};
  const int st = g.stride;
  a.src = dy; a.wgt = wt;
  a.Hs = g.P; a.Ws = g.Q; a.Cs = g.K; a.Ng = g.C;
  a.ldb = (long)g.R * g.S * g.K;
  a.stride = 1; a.base_h = 0; a.base_w = 0;
  a.P = (g.H - ph + st - 1) / st;
  a.Q = (g.W - pw + st - 1) / st;
  a.M = g.N * a.P * a.Q;
  if (st > 1) {
    a.omap = 1; a.oH = g.H; a.oW = g.W; a.osh = st; a.osw = st; a.ooh = ph; a.oow = pw;
  }
  int n = 0;
  for (int r = 0; r < g.R; ++r) {
    if (((ph + g.pad - r) % st + st) % st) continue;
    for (int q = 0; q < g.S; ++q) {
      if (((pw + g.pad - q) % st + st) % st) continue;
      if (n == 9) { a.ntaps = 0; cd_divs(a); return a; }
      a.tap_dh[n] = (ph + g.pad - r) / st;
      a.tap_dw[n] = (pw + g.pad - q) / st;
      a.tap_kcol[n] = (r * g.S + q) * g.K;
      ++n;
    }
  }
  a.ntaps = n;
  a.Kd = n * g.K;
  cd_divs(a);
  return a;
}

// ===========================================================================
// LDS-DMA conv weight gradient (split over output pixels, fp32 atomics)
//
//   dW[k][(r,s,c)] = sum_m dY[m][k] * X[n, p*st-pad+r, q*st-pad+s, c],  m = (n,p,q)
//
// GEMM rows = k (BM), cols = (r,s,c) (BN), reduction = m in 64-pixel steps.
// BN divides C, so a column tile is ONE tap (r,s) and BN channels: each
// pixel row of the B tile is one contiguous BN*2-byte segment of X (or the
// zero row for a padding tap / the pixel tail), each row of the A tile a
// contiguous BM*2-byte segment of dY. Both images are [64 pixels][cols]
// (pixel-major), kept as 64 x min(cols,128) sub-images with the MN-major
// swizzle of igemm.h (applied on the DMA source chunk) and read with
// ds_read_b64_tr_b16 (read_frag_mn). Each thread advances its rows' (n,p,q)
// incrementally (no per-step division); the split's blocks accumulate into
// the fp32 dW with no-return float atomics.
// ===========================================================================
struct WGArgs {
  const bf16_t* dy;    // [Mred][K]
  const bf16_t* x;     // NHWC [N][H][W][C]
  float* dw;           // [K][R*S*C]
  long ldc;            // R*S*C
  int K, C, H, W, P, Q, S, stride, pad;
  int Mred;            // N*P*Q
  int steps_per_split; // 64-pixel steps per blockIdx.z
  int dn, dp, dq;      // 64 pixels = dn images + dp rows + dq columns
  int atomic;          // 1: atomic add, 0: plain += (single split)
  float* dbias;        // optional: dbias[k] += sum_m dY[m][k] (the conv's bias gradient)
  int tiles;           // output tiles per split
  int flat;            // 1: 1-D grid of tiles x splits, split-major per XCD (see below)
  float* slab;         // split-K partials [splits][K][ldc], plain stores (nullptr: atomics into dw)
};

template <int S>
__device__ __forceinline__ int wg_swz16(int row) { return mnmaj_swz<S>(row) >> 1; }

template <int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(64 * WM * WN, 1) conv_wgrad_dma_kernel(WGArgs a) {
  constexpr int W = WM * WN, BK = 64;
  constexpr int SA = BM < 128 ? BM : 128, SB = BN < 128 ? BN : 128;   // sub-image widths
  constexpr int A_BYTES = BK * BM * 2, B_BYTES = BK * BN * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int STAGES = 3 * STAGE <= 160 * 1024 ? 3 : 2;
  constexpr int AI = BM / 8 / W, BI = BN / 8 / W;   // DMA instructions per thread per step
  constexpr int D = AI + BI;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  static_assert(AI >= 1 && BI >= 1 && BM % (8 * W) == 0 && BN % (8 * W) == 0, "tile/wave split");
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % WM, wn = wid / WM;
  const int tiles_m = (a.K + BM - 1) / BM;
  const int ncols = (int)a.ldc;
  const int tiles_n = ncols / BN;
  // Block -> (tile, split). The hardware deals workgroups round-robin over
  // the 8 XCDs by LINEAR id; a (tiles, 1, splits) grid remapped on x alone
  // spreads every split's pixel rows over all 8 L2s, and each XCD's working
  // set is the whole dY + X (12.8 MB at 14x14x256, 4 MB of L2). The flat
  // form remaps the linear id so each XCD owns a run of consecutive splits
  // with all their tiles: one split's dY rows are fetched into one L2 and
  // shared by every column tile, its X rows by every row tile.
  int bid, split;
  if (a.flat) {
    const int f = xcd_remap(blockIdx.x, gridDim.x);
    bid = f % a.tiles; split = f / a.tiles;
  } else {
    bid = xcd_remap(blockIdx.x, gridDim.x); split = blockIdx.z;
  }
  const int tm = bid % tiles_m, tn = bid / tiles_m;
  const int k0 = tm * BM, col0 = tn * BN;
  (void)tiles_n;
  // this column tile's tap and channel offset
  const int rs = col0 / a.C, c0 = col0 % a.C;
  const int tr = rs / a.S, ts = rs % a.S;

  const int step0 = split * a.steps_per_split;
  const int nsteps_all = (a.Mred + BK - 1) / BK;
  const int nk = min(a.steps_per_split, nsteps_all - step0);
  const int mstart = step0 * BK;

  // ---- A rows (dY): instruction g -> sub-image h, rows RPI*li + lane/(SA/8)
  constexpr int LPR_A = SA / 8, RPI_A = 64 / LPR_A;
  const bf16_t* aptr[AI];
  int arow[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int g = wid + W * j;
    const int h = g / (SA / 8), li = g % (SA / 8);
    const int row = RPI_A * li + lane / LPR_A;
    const int lc = (lane % LPR_A) ^ wg_swz16<SA>(row);
    int k = k0 + h * SA + 8 * lc;
    k = k < a.K ? k : a.K - 8;             // clamp: rows of dW past K are never stored
    arow[j] = row;
    aptr[j] = a.dy + (long)(mstart + row) * a.K + k;
  }
  // ---- B rows (X): per row the pixel (n,p,q) of m = mstart + row, advanced per step
  constexpr int LPR_B = SB / 8, RPI_B = 64 / LPR_B;
  int bn_[BI], bp_[BI], bq_[BI], bcol[BI], brow[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int g = wid + W * j;
    const int h = g / (SB / 8), li = g % (SB / 8);
    const int row = RPI_B * li + lane / LPR_B;
    const int lc = (lane % LPR_B) ^ wg_swz16<SB>(row);
    brow[j] = row;
    bcol[j] = c0 + h * SB + 8 * lc;
    const int m = mstart + row;
    const int q = m % a.Q, t = m / a.Q;
    bq_[j] = q; bp_[j] = t % a.P; bn_[j] = t / a.P;
  }
  const bf16_t* zero = g_cd_zero;

  auto issue = [&](int step, int st) {
    char* sa = smem + st * STAGE;
    char* sb = sa + A_BYTES;
    const int mb = mstart + step * BK;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int g = wid + W * j;
      const int h = g / (SA / 8), li = g % (SA / 8);
      const bool ok = mb + arow[j] < a.Mred;
      const bf16_t* p = ok ? aptr[j] + (long)step * BK * a.K : zero + 8 * (lane % LPR_A);
      __builtin_amdgcn_global_load_lds((const void*)p,
                                       (cd_lds_void_t*)(sa + h * (BK * SA * 2) + li * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const int g = wid + W * j;
      const int h = g / (SB / 8), li = g % (SB / 8);
      const int hh = bp_[j] * a.stride - a.pad + tr, ww = bq_[j] * a.stride - a.pad + ts;
      const bool ok = mb + brow[j] < a.Mred && (unsigned)hh < (unsigned)a.H &&
                      (unsigned)ww < (unsigned)a.W;
      const bf16_t* p = ok ? a.x + ((long)(bn_[j] * a.H + hh) * a.W + ww) * a.C + bcol[j]
                           : zero + 8 * (lane % LPR_B);
      __builtin_amdgcn_global_load_lds((const void*)p,
                                       (cd_lds_void_t*)(sb + h * (BK * SB * 2) + li * 1024), 16, 0, 0);
      // advance this row's pixel by 64
      int q = bq_[j] + a.dq, pp = bp_[j] + a.dp, n = bn_[j] + a.dn;
      if (q >= a.Q) { q -= a.Q; ++pp; }
      if (pp >= a.P) { pp -= a.P; ++n; }
      bq_[j] = q; bp_[j] = pp; bn_[j] = n;
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // fused bias gradient: the column-tile-0 blocks' wn == 0 waves add up the
  // dY fragments they already read (lane: 8 pixels of channel 16i + lane%16)
  const bool bsum_on = a.dbias != nullptr && tn == 0 && wn == 0;
  float bsum[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) bsum[i] = 0.f;

  if (nk > 0) {
#pragma unroll
    for (int t = 0; t < STAGES - 1; ++t)
      if (t < nk) issue(t, t);
    for (int t = 0; t < nk; ++t) {
      if constexpr (STAGES == 3) {
        if (t + 1 < nk) cd_vm_wait<D>();
        else cd_vm_wait<0>();
      } else {
        cd_vm_wait<0>();
      }
      cd_barrier();
      if (t + STAGES - 1 < nk) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
      const char* ta = smem + (t % STAGES) * STAGE;
      const char* tb = ta + A_BYTES;
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        s16x8_t fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int c = wm * (BM / WM) + 16 * i;
          fa[i] = read_frag_mn<SA>(ta + (c / SA) * (BK * SA * 2), lane, 32 * kk, c % SA);
        }
        if (bsum_on) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int e = 0; e < 8; ++e) bsum[i] += __uint_as_float((uint32_t)(uint16_t)fa[i][e] << 16);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int c = wn * (BN / WN) + 16 * j;
          fb[j] = read_frag_mn<SB>(tb + (c / SB) * (BK * SB * 2), lane, 32 * kk, c % SB);
        }
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

  if (bsum_on) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float v = bsum[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int k = k0 + wm * (BM / WM) + 16 * i + lane;
      if (lane < 16 && k < a.K) atomicAdd(a.dbias + k, v);
    }
  }
  // ---- epilogue: row = k, col = (r,s,c); fp32 accumulate into dW, or store
  // this split's partial tile into its slab (reduced by gemm_slab_reduce)
  float* slab = a.slab ? a.slab + (long)split * a.K * a.ldc : nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col0 + wn * (BN / WN) + 16 * j + (lane & 15);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = k0 + wm * (BM / WM) + 16 * i + 4 * (lane >> 4) + r;
        if (row >= a.K) continue;
        const long off = (long)row * a.ldc + col;
        if (slab) slab[off] = acc[i][j][r];
        else if (a.atomic) atomicAdd(a.dw + off, acc[i][j][r]);
        else a.dw[off] += acc[i][j][r];
      }
    }
  }
}

// ===========================================================================
// Weight gradient of a 3x3 stride-1 "same" conv, per 64-channel input slice
// (VGG-16's 224x224 / 112x112 layers, ResNet-50's 56x56 stage): dW is only
// K x 576 but the pixel reduction is 0.2-1.6 M long, and the tap-gather
// cores re-read X nine times through L2 (202 TF/s on VGG's first wgrad).
// Here a block owns a 64-channel k-slice x 64-channel input slice (grid y,
// z) and sweeps 112-pixel tiles (half a
// 224 row, a 112 row, or two 56 rows): per tile the dY rows (128-row image,
// 112 live) and the X PATCH with its halo ((rows+2) x (cols+2) pixels x 64
// channels, zero padded) are staged ONCE by LDS-DMA, and every tap's B
// fragment is a per-lane-group shifted read of the patch (8-pixel groups
// never straddle an image row). Wave w owns N-tiles 9w..9w+8 of the 36
// (tap, 16-channel) tiles and all four 16-k tiles: 144 fp32 accumulators per
// lane, one dY fragment per k-tile reused across its 9 B fragments. At the
// end every accumulator is added into the fp32 dW (no-return atomics).
// ===========================================================================
constexpr int WC_TP = 112;                    // live pixels per tile
constexpr int WC_ROWS = 128;                  // dY image rows (4 chunks of 32)
// patch rows, largest tile shape (3 x 114 = 342) rounded up to the 8-row
// (1 KiB) DMA granule: the last DMA group of a patch writes whole 1-KiB
// blocks, which at 342 rows spilled into the other buffer's dY image
constexpr int WC_MAXP = 344;

struct WCArgs {
  const bf16_t* dy;    // [N][H][W][K]
  const bf16_t* x;     // [N][H][W][C]
  float* dw;           // [K][3][3][C]
  int N, H, W, K, C;   // C % 64 == 0: blockIdx.z = 64-channel input slice
  int tw, tr;          // tile: tr image rows x tw columns (tr * tw == 112)
  int ntiles;
  float* dbias;        // optional: dbias[k] += sum dY[.][k] (input slice 0, wave 0)
};

// MN-major transposed fragment read whose 8 rows for this lane group start
// at `rbase` (a per-group base instead of kbase + 8g; read_frag_mn's layout)
__device__ __forceinline__ s16x8_t wc_frag(const char* tile, int lane, int rbase, int colbase) {
  const int t = lane & 15, q = t >> 2, p = t & 3;
  const int c8 = (colbase >> 2) + p;
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + mnmaj_off<64>(rbase + q, c8)));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + mnmaj_off<64>(rbase + q + 4, c8)));
  s16x8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

static __global__ void __launch_bounds__(256, 1) conv_wgrad_c64_kernel(WCArgs a) {
  // two buffers of [dY image | X patch]: tile t+grid's DMA lands while tile t computes
  constexpr int BUF = WC_ROWS * 128 + WC_MAXP * 128;
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int kb = blockIdx.y * 64, cb = blockIdx.z * 64;
  const int pw = a.tw + 2, npat = (a.tr + 2) * pw;
  const int tq = a.W / a.tw, th = a.H / a.tr;
  f32x4_t acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // fused bias gradient from the dY fragments wave 0 of input slice 0 reads
  const bool bsum_on = a.dbias != nullptr && blockIdx.z == 0 && w == 0;
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int tile, char* buf) {
    char* dyi = buf;
    char* pat = buf + WC_ROWS * 128;
    const int qb = tile % tq, rest = tile / tq;
    const int hb = rest % th, n = rest / th;
    const int h0 = hb * a.tr, q0 = qb * a.tw;
    // dY image: row i = tile pixel i (rows >= 112 zero); the granule for
    // LDS slot `slot` of row i is source granule slot ^ swz(i) (the DMA
    // writes lane-linear: the swizzle goes on the source)
#pragma unroll
    for (int j = 0; j < WC_ROWS * 8 / 256; ++j) {
      const int gi = j * 256 + tid;
      const int row = gi >> 3, slot = gi & 7;
      const int c = slot ^ (mnmaj_swz<64>(row) >> 1);
      const bf16_t* src = g_cd_zero + 8 * c;
      if (row < WC_TP) {
        const int hh = h0 + row / a.tw, qq = q0 + row % a.tw;
        src = a.dy + (((long)n * a.H + hh) * a.W + qq) * a.K + kb + 8 * c;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (cd_lds_void_t*)(dyi + (gi >> 6) * 1024), 16, 0, 0);
    }
    // X patch: row r = pixel (h0 - 1 + r / pw, q0 - 1 + r % pw), zero outside
    for (int gi = tid; gi < ((npat * 8 + 63) & ~63); gi += 256) {
      const int row = gi >> 3, slot = gi & 7;
      const int c = slot ^ (mnmaj_swz<64>(row) >> 1);
      const bf16_t* src = g_cd_zero + 8 * c;
      if (row < npat) {
        const int hh = h0 - 1 + row / pw, qq = q0 - 1 + row % pw;
        if ((unsigned)hh < (unsigned)a.H && (unsigned)qq < (unsigned)a.W)
          src = a.x + (((long)n * a.H + hh) * a.W + qq) * a.C + cb + 8 * c;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (cd_lds_void_t*)(pat + (gi >> 6) * 1024), 16, 0, 0);
    }
  };

  if (blockIdx.x < a.ntiles) stage(blockIdx.x, smem);
  int it = 0;
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x, ++it) {
    char* buf = smem + (it & 1) * BUF;
    cd_vm_wait<0>();                 // this tile's DMA (issued one iteration ago) landed ...
    cd_barrier();                    // ... for every wave; and all are done with the other buffer
    if (tile + (int)gridDim.x < a.ntiles) stage(tile + gridDim.x, smem + ((it + 1) & 1) * BUF);
    const char* dyi = buf;
    const char* pat = buf + WC_ROWS * 128;
#pragma unroll
    for (int ch = 0; ch < WC_ROWS / 32; ++ch) {
      // this lane group's 8 pixels: tile pixel i0 = 32ch + 8g (clamped past 112;
      // their dY rows are zero)
      int i0 = 32 * ch + 8 * g;
      i0 = i0 < WC_TP ? i0 : 0;
      const int pbase = (i0 / a.tw) * pw + (i0 % a.tw);   // patch row at tap (0, 0)
      s16x8_t fa[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) fa[kt] = read_frag_mn<64>(dyi, lane, 32 * ch, 16 * kt);
      if (bsum_on) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int e = 0; e < 8; ++e) bsum[kt] += __uint_as_float((uint32_t)(uint16_t)fa[kt][e] << 16);
      }
#pragma unroll
      for (int nn = 0; nn < 9; ++nn) {
        const int nt = 9 * w + nn, tap = nt >> 2, ct = nt & 3;
        const int dh = tap / 3, dwc = tap % 3;
        const s16x8_t fb = wc_frag(pat, lane, pbase + dh * pw + dwc, 16 * ct);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
          acc[kt][nn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[kt]),
                                                                __builtin_bit_cast(bf16x8_t, fb), acc[kt][nn], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }
  if (bsum_on) {
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      float v = bsum[kt];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) atomicAdd(a.dbias + kb + 16 * kt + lane, v);
    }
  }
  // ---- dW[kb + 16kt + 4g' + r][tap][16ct + (lane&15)] += acc
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int nn = 0; nn < 9; ++nn) {
      const int nt = 9 * w + nn, tap = nt >> 2, ct = nt & 3;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = kb + 16 * kt + 4 * (lane >> 4) + r;
        unsafeAtomicAdd(a.dw + (long)k * 9 * a.C + tap * a.C + cb + 16 * ct + (lane & 15), acc[kt][nn][r]);
      }
    }
}

// dW (+)= wgrad of a 3x3 / stride 1 / pad 1 conv over a 64-channel input on
// conv_wgrad_c64_kernel; false when the shape is not for it
// force_small: also the 56-wide grids (two-row tiles), measured slower than
// the tap-gather path on ResNet-50's stage 1 (tests / A/B only)
inline bool launch_conv_wgrad_c64(const bf16_t* dy, const bf16_t* x, float* dw, const ConvGeom& g, int mode,
                                  int blocks_per_kslice, hipStream_t s, bool force_small = false,
                                  float* dbias = nullptr) {
  if (g.C % 64 != 0 || g.R != 3 || g.S != 3 || g.stride != 1 || g.pad != 1 || g.dil != 1 || g.K % 64 != 0)
    return false;
  if (g.C != 64 && !force_small) return false;   // wider inputs (channel slices): tests / A/B until measured
  if (g.P != g.H || g.Q != g.W) return false;
  int tw, tr;
  if (g.W % 112 == 0) { tw = 112; tr = 1; }
  else if (g.W == 56 && force_small) { tw = 56; tr = 2; }   // (ResNet's 56x56: 74 vs 61 us on the tap-gather path)
  else return false;
  if (g.H % tr != 0 || (long)g.N * g.H * g.W * (g.K > g.C ? g.K : g.C) >= (1L << 31)) return false;
  if ((((tr + 2) * (tw + 2) + 7) & ~7) > WC_MAXP) return false;   // patch DMA groups must fit the buffer
  const int ntiles = g.N * (g.H / tr) * (g.W / tw);
  if (mode == 0) zero_async(dw, (size_t)g.K * 9 * g.C * sizeof(float), s);
  WCArgs a{dy, x, dw, g.N, g.H, g.W, g.K, g.C, tw, tr, ntiles, dbias};
  const int slices = (g.K / 64) * (g.C / 64);
  int bx = blocks_per_kslice > 0 ? blocks_per_kslice : 256 / slices;   // one block per CU
  if (bx < 1) bx = 1;
  if (bx > ntiles) bx = ntiles;
  hipLaunchKernelGGL(conv_wgrad_c64_kernel, dim3(bx, g.K / 64, g.C / 64), dim3(256), 0, s, a);
  return true;
}

// (bm, bn, splits) forced for A/B sweeps (tools/sweep_wgrad.py); 0 = the
// heuristic below. [3] != 0: TIMING ONLY -- split blocks add with plain
// (racy) read-modify-writes instead of atomics, to price the atomic traffic
inline int g_wgrad_force[4] = {0, 0, 0, 0};
// block order of the DMA wgrad kernel: 1 split-major flat XCD remap
// (default), 0 the (tiles, 1, splits) grid (A/B: conv_wgrad_order)
inline int g_wgrad_flat = 1;

template <int BM, int BN, int WM, int WN>
inline void wgrad_dma_launch(const WGArgs& a, int tiles, int splits, hipStream_t s) {
  const dim3 grid = a.flat ? dim3(tiles * splits) : dim3(tiles, 1, splits);
  hipLaunchKernelGGL((conv_wgrad_dma_kernel<BM, BN, WM, WN>), grid, dim3(64 * WM * WN), 0, s, a);
}

// slab split-K for the DMA wgrad: 1 (default) split passes store fp32
// partials and one reduce pass adds them into dw (store mode needs no zero
// pass); 0: every split adds into dw with fp32 atomics (A/B). The atomics /
// read-modify-writes of the split epilogues run at ~1.2 TB/s chip-wide
// (32 MB of them at 256 blocks of 256x128: ~27 us on ResNet-50's 14x14
// layers), the slab's plain stores + one streaming reduce at HBM rate.
inline int g_wgrad_slab = 1;

struct WGPlan {
  int bm = 0, bn = 0, tiles = 0, splits = 0, sps = 0;
  bool ok = false;
};

inline WGPlan wgrad_dma_plan(const ConvGeom& g, bool force) {
  WGPlan p;
  if (g.dil != 1 || g.C % 64 != 0 || g.K % 64 != 0) return p;
  const long Mred = (long)g.N * g.P * g.Q;
  if (Mred >= (1L << 31) || (long)g.N * g.H * g.W * g.C >= (1L << 31)) return p;
  const int ncols = g.R * g.S * g.C;
  // tile: BN divides C (one tap per column tile); BM over K.
  // 1x1 wgrads over >= 100K pixels (ResNet-50's 56x56 stage) stream dY and X
  // from HBM: small tiles at two blocks per CU hide more latency than big
  // tiles at one (64->256: 47 -> 32 us, 256->64: 49 -> 34 us, 256->128:
  // 51 -> 45 us; profiles/r4/wgrad_sweep_56.json)
  // The same holds for 3x3 wgrads over >= 256K pixels with K % 128 == 0
  // (VGG-16's 112x112 128->128: 322 -> 264 us at 128x64 / 28 splits;
  // profiles/r4/wgrad_sweep_vgg.json); the 56x56 VGG layers stay on 256x128.
  // 64->64 3x3 over >= 1M pixels (VGG-16's 224x224 layer when it runs on
  // the weight-gradient side stream, where the patch kernel is not used):
  // 64x64 tiles at 256 splits, 580 (igemm) -> 343 us
  // (profiles/r4/wgrad_sweep_vgg224.json).
  const bool stream = (g.R == 1 && g.S == 1 && Mred >= 100352) || (Mred >= 262144 && g.K % 128 == 0) ||
                      (Mred >= (1L << 20) && g.K == 64);
  const int* fw = g_wgrad_force;
  if (fw[0] > 0) {
    p.bm = fw[0]; p.bn = fw[1];
    const bool known = (p.bm == 256 && (p.bn == 128 || p.bn == 64)) || (p.bm == 128 && (p.bn == 128 || p.bn == 64)) ||
                       (p.bm == 64 && p.bn == 64);
    if (!known || g.K % p.bm != 0 || g.C % p.bn != 0) return p;
  } else if (stream) {
    p.bm = g.K % 128 == 0 ? 128 : 64; p.bn = 64;
  } else {
    if (g.K % 256 == 0 && g.C % 128 == 0) { p.bm = 256; p.bn = 128; }
    else if (g.K % 128 == 0 && g.C % 128 == 0) { p.bm = 128; p.bn = 128; }
    else { p.bm = 64; p.bn = 64; }
    // the 64x64 form beats the igemm only on 1x1 layers (measured)
    if (!force && p.bm == 64 && !(g.R == 1 && g.S == 1)) return p;
  }
  p.tiles = (g.K / p.bm) * (ncols / p.bn);
  const int nsteps = (int)((Mred + 63) / 64);
  // split the pixel reduction to ~one block per CU (two for the streaming
  // 1x1 passes, whose small tiles leave room for a second block), not
  // more: every split adds |dW| of fp32 partials to write and reduce
  const int target = !stream ? 256 : (p.bm == 64 && !(g.R == 1 && g.S == 1) ? 2304 : 512);
  int splits = fw[2] > 0 ? fw[2] : target / p.tiles;
  if (fw[2] <= 0 && splits > nsteps / 8) splits = nsteps / 8;
  if (splits > nsteps) splits = nsteps;
  if (splits < 1) splits = 1;
  p.sps = (nsteps + splits - 1) / splits;
  p.splits = (nsteps + p.sps - 1) / p.sps;
  p.ok = true;
  return p;
}

// fp32 slab floats launch_conv_wgrad_dma would use for this geometry (0: none)
inline long wgrad_dma_slab_floats(const ConvGeom& g, bool force) {
  if (!g_wgrad_slab || g_wgrad_force[3]) return 0;
  const WGPlan p = wgrad_dma_plan(g, force);
  if (!p.ok || p.splits < 2) return 0;
  return (long)p.splits * g.K * g.R * g.S * g.C;
}

// dw = (mode ? dw : 0) + conv wgrad
// ws / ws_floats: slab scratch of wgrad_dma_slab_floats(g) floats (else atomics)
// slab_defer (non-null): a slab launch leaves the reduce to the caller and
// reports its slab count there (*slab_defer = splits; 0: nothing deferred)
inline bool launch_conv_wgrad_dma(const bf16_t* dy, const bf16_t* x, float* dw, const ConvGeom& g,
                                  int mode, hipStream_t s, bool force = false, float* dbias = nullptr,
                                  float* ws = nullptr, long ws_floats = 0, int* slab_defer = nullptr) {
  const WGPlan p = wgrad_dma_plan(g, force);
  if (!p.ok) return false;
  const int ncols = g.R * g.S * g.C;
  const bool slab = p.splits > 1 && ws != nullptr && ws_floats >= wgrad_dma_slab_floats(g, force) &&
                    wgrad_dma_slab_floats(g, force) > 0;
  if (mode == 0 && !slab) zero_async(dw, (size_t)g.K * ncols * sizeof(float), s);
  const int PQ = g.P * g.Q;
  WGArgs a{dy, x, dw, ncols, g.K, g.C, g.H, g.W, g.P, g.Q, g.S, g.stride, g.pad, g.N * g.P * g.Q, p.sps,
           64 / PQ, (64 % PQ) / g.Q, (64 % PQ) % g.Q, p.splits > 1 && !g_wgrad_force[3] ? 1 : 0, dbias,
           p.tiles, g_wgrad_flat, slab ? ws : nullptr};
  const int bm = p.bm, bn = p.bn;
  if (bm == 256 && bn == 128) wgrad_dma_launch<256, 128, 4, 2>(a, p.tiles, p.splits, s);
  else if (bm == 256) wgrad_dma_launch<256, 64, 4, 1>(a, p.tiles, p.splits, s);
  else if (bm == 128 && bn == 128) wgrad_dma_launch<128, 128, 2, 2>(a, p.tiles, p.splits, s);
  else if (bm == 128) wgrad_dma_launch<128, 64, 2, 2>(a, p.tiles, p.splits, s);
  else wgrad_dma_launch<64, 64, 2, 2>(a, p.tiles, p.splits, s);
  if (slab && slab_defer) *slab_defer = p.splits;
  else if (slab) wgrad_slab_reduce(ws, p.splits, (long)g.K * ncols, dw, mode, s);
  return true;
}

}  // namespace tam
