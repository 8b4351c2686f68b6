// tiresias_amd — skinny-M weight-streaming GEMM (M <= 64): the VGG
// classifier's batch-32 Linear layers, forward (C = x W^T, W [N][K] K-major)
// and input gradient (dX = dY W, W [K][N] N-major).
//
//   C[M][N] (op)= alpha * A[M][K] . B(k,n) (+bias)(relu)(mask)
//
// At M = 32 the weight is read once and each element feeds only 32 MACs:
// the op is an HBM stream of the weight (205 MB for 32x4096x25088), not an
// MFMA problem. The square-tile kernels waste 3/4 of their tile on padding
// rows and leave the chip underfilled (146 us vs ~30-40 us streaming time,
// VERDICT r3 item 7a). MI355X-first structure:
//  * block = 4 waves, a 128-column slice of W x ALL M rows (MT x 16, MT = 2
//    or 4) x a K-slice; grid = column slices x K-slices sized to ~one block
//    per CU (split-K), so every CU streams its share of W.
//  * W and x tiles (BK = 64) go HBM/L2 -> LDS by LDS-DMA
//    (global_load_lds_dwordx4, no VGPR round trip) into an NST-deep ring:
//    NST-1 tiles in flight per block, one counted vmcnt + one raw s_barrier
//    per K-tile. K-major images use the (row>>1)&7 chunk swizzle
//    (read_frag_k, ds_read_b128); the N-major W image is [64 k][128 n] read
//    with the ds_read_b64_tr_b16 transpose (read_frag_mn) -- both swizzles
//    applied to the per-lane SOURCE address (guide rule 21).
//  * x (L2-resident, re-read by every column slice) is the MFMA A operand,
//    W the B operand: 16x16x32 bf16 MFMAs, acc[MT][2] per wave.
//  * blockIdx -> (K-slice, column slice) after the bijective XCD remap (T1):
//    consecutive ids on one XCD share a K-slice, so its x panel stays in
//    that XCD's L2.
//  * split-K partials go to an fp32 slab ws[sp][M][N]; the slab reduce
//    (gemm.hip) applies the epilogue. One slice writes C directly.
#include "tam/launch.h"
#include "tam/tiles.h"

namespace tam {

constexpr int SK_BN = 128, SK_BK = 64;
typedef __attribute__((address_space(3))) void sk_lds_t;

struct SkArgs {
  const bf16_t* A;   // [M][lda] K-major
  long lda;
  const bf16_t* B;   // [N][ldb] K-major (BK) or [K][ldb] N-major
  long ldb;
  int M, N, K;
  int kps;           // K-tiles per slice
  int ntile;         // column slices
  float* ws;         // slab base (sp > 1) or null
};

__device__ __forceinline__ void sk_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int MT, bool BK, int NST>
__global__ void __launch_bounds__(256, 2) gemm_skinny_kernel(SkArgs a, Epi ep) {
  constexpr int XB = MT * 16 * SK_BK * 2;          // x image bytes
  constexpr int WB = SK_BN * SK_BK * 2;            // W image bytes (16 KiB)
  constexpr int STAGE = WB + XB;
  constexpr int XG = XB / 1024 / 4;                // x DMA groups per wave
  constexpr int PER_TILE = 4 + XG;                 // DMA instructions per thread per K-tile
  __shared__ __attribute__((aligned(1024))) char smem[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kz = bid / a.ntile, tn = bid % a.ntile;
  const int n0 = tn * SK_BN;
  const int ktiles = a.K / SK_BK;
  const int kt0 = kz * a.kps;
  const int nk = min(ktiles, kt0 + a.kps) - kt0;

  auto issue = [&](int t) {
    char* st = smem + (t % NST) * STAGE;
    const int k0 = (kt0 + t) * SK_BK;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int g = j * 4 + wid;                   // 1-KiB group of the W image
      if constexpr (BK) {
        const int lr = g * 8 + (lane >> 3);        // 8 rows x 128 B per group
        const int c = (lane & 7) ^ ((lr >> 1) & 7);
        int r = n0 + lr;
        r = r < a.N ? r : a.N - 1;                 // columns past N are never stored
        __builtin_amdgcn_global_load_lds((const void*)(a.B + (long)r * a.ldb + k0 + c * 8),
                                         (sk_lds_t*)(st + g * 1024), 16, 0, 0);
      } else {
        const int kr = g * 4 + (lane >> 4);        // 4 k-rows x 256 B per group
        const int gran = (lane & 15) ^ (mnmaj_swz<SK_BN>(kr) >> 1);
        int col = n0 + gran * 8;
        col = col + 8 <= a.N ? col : a.N - 8;      // N % 8 == 0
        __builtin_amdgcn_global_load_lds((const void*)(a.B + (long)(k0 + kr) * a.ldb + col),
                                         (sk_lds_t*)(st + g * 1024), 16, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < XG; ++j) {
      const int g = j * 4 + wid;
      const int lr = g * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((lr >> 1) & 7);
      const int r = lr < a.M ? lr : a.M - 1;       // rows past M are never stored
      __builtin_amdgcn_global_load_lds((const void*)(a.A + (long)r * a.lda + k0 + c * 8),
                                       (sk_lds_t*)(st + WB + g * 1024), 16, 0, 0);
    }
  };

  f32x4_t acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) issue(s);
  for (int t = 0; t < nk; ++t) {
    // tile t landed (this thread's DMAs), tiles t+1 .. t+NST-2 may fly
    const int ahead = min(nk - 1 - t, NST - 2);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_TILE) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_TILE) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sk_barrier();   // every thread's part of tile t is in LDS; tile t-1's readers are done
    if (t + NST - 1 < nk) issue(t + NST - 1);     // refills tile t-1's stage
    const char* st = smem + (t % NST) * STAGE;
    s16x8_t fa[MT][2], fb[2][2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (BK) fb[j][kk] = read_frag_k(st, lane, wid * 32 + 16 * j, kk);
        else fb[j][kk] = read_frag_mn<SK_BN>(st, lane, 32 * kk, wid * 32 + 16 * j);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) fa[i][kk] = read_frag_k(st + WB, lane, 16 * i, kk);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[i][kk]),
                                                              __builtin_bit_cast(bf16x8_t, fb[j][kk]),
                                                              acc[i][j], 0, 0, 0);
  }

  // C/D map of 16x16x32: col = lane&15 (n), row = 4*(lane>>4) + r (m)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wid * 32 + 16 * j + (lane & 15);
    if (col >= a.N) continue;
    const float bv = (ep.bias && !a.ws) ? bf2f(ep.bias[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * i + 4 * (lane >> 4) + r;
        if (row >= a.M) continue;
        if (a.ws) {                                 // split-K slab: raw partial sums
          a.ws[((long)kz * a.M + row) * a.N + col] = acc[i][j][r];
          continue;
        }
        float v = acc[i][j][r] * ep.alpha + bv;
        if (ep.relu) v = fmaxf(v, 0.f);
        if (ep.mask && bf2f(ep.mask[(long)row * ep.ldm + col]) <= 0.f) v = 0.f;
        const long off = (long)row * ep.ldc + col;
        if (ep.c_f32) {
          float* c = (float*)ep.c;
          if (ep.mode == 2) atomicAdd(c + off, v);
          else c[off] = ep.mode == 1 ? c[off] + v : v;
        } else {
          bf16_t* c = (bf16_t*)ep.c;
          c[off] = f2bf(ep.mode == 1 ? v + bf2f(c[off]) : v);
        }
      }
  }
}

static int g_sk_policy = 1, g_sk_force_sp = 0, g_sk_nst = 3;
TAM_KNOB(g_sk_policy) TAM_KNOB(g_sk_force_sp) TAM_KNOB(g_sk_nst)
void gemm_skinny_policy(int on, int force_splits, int nst) {
  g_sk_policy = on;
  g_sk_force_sp = force_splits > 0 ? force_splits : 0;
  g_sk_nst = nst == 4 ? 4 : 3;
}

bool gemm_skinny_ok(bool ak, bool bk, int M, int N, int K, long lda, long ldb) {
  if (!g_sk_policy || !ak || M < 1 || M > 64 || N < 128) return false;
  if (K % SK_BK != 0 || K < 2 * SK_BK || lda % 8 != 0 || ldb % 8 != 0) return false;
  if (!bk && N % 8 != 0) return false;
  return true;
}

int gemm_skinny_splits(int M, int N, int K) {
  const int ntile = cdiv(N, SK_BN), kt = K / SK_BK;
  if (N % 4 != 0) return 1;                        // the slab reduce's float4 rows
  int sp = g_sk_force_sp;
  if (!sp) {
    // ~one block per CU and >= 8 K-tiles per slice: more slices only add
    // slab-reduce traffic (M N sp fp32) -- measured best-or-within-5 % on
    // every VGG classifier shape (tools/bench_skinny.py, profiles/r4/skinny.json)
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      TAM_HIP_CHECK(hipGetDevice(&dev));
      TAM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      if (cus < 1) cus = 256;
    }
    sp = (cus + ntile - 1) / ntile;
    if (sp > kt / 8) sp = kt / 8;
    if (sp > 64) sp = 64;
  }
  if (sp < 1) sp = 1;
  const int kps = cdiv(kt, sp);
  return cdiv(kt, kps);                            // slices actually launched
}

template <int MT, bool BK>
static void sk_launch_mt(const SkArgs& g, const Epi& ep, dim3 grid, hipStream_t s) {
  if (g_sk_nst == 4) hipLaunchKernelGGL((gemm_skinny_kernel<MT, BK, 4>), grid, dim3(256), 0, s, g, ep);
  else hipLaunchKernelGGL((gemm_skinny_kernel<MT, BK, 3>), grid, dim3(256), 0, s, g, ep);
}

void gemm_skinny(const bf16_t* A, long lda, const bf16_t* B, long ldb, bool bk, int M, int N, int K,
                 const Epi& ep, int sp, float* ws, hipStream_t s) {
  const int kt = K / SK_BK;
  const int kps = cdiv(kt, sp < 1 ? 1 : sp);
  const int z = cdiv(kt, kps);
  SkArgs g{A, lda, B, ldb, M, N, K, kps, cdiv(N, SK_BN), z > 1 ? ws : nullptr};
  const dim3 grid((unsigned)(g.ntile * z));
  if (M <= 32) {
    if (bk) sk_launch_mt<2, true>(g, ep, grid, s);
    else sk_launch_mt<2, false>(g, ep, grid, s);
  } else {
    if (bk) sk_launch_mt<4, true>(g, ep, grid, s);
    else sk_launch_mt<4, false>(g, ep, grid, s);
  }
  if (z > 1) gemm_slab_reduce(ws, z, M, N, ep, s);
}

}  // namespace tam
