// tiresias_amd — MFMA GEMM entry points (all four operand majorities) and the
// tile / split-K selection heuristic shared with the conv passes.
#include "tam/launch.h"
#include "tam/tiles.h"
#include "tam/gemm256.h"
#include "tam/gemm8p.h"
#include "tam/gemm_dma.h"

namespace tam {

template <int BM, int BN, int NPF>
static void gemm_tile_p(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk,
                        int M, int N, int K, Epi ep, int splits, hipStream_t s) {
  if (ak && bk) {
    LdKMajor<BM> la{A, lda, M, K}; LdKMajor<BN> lb{B, ldb, N, K};
    launch_igemm<BM, BN, NPF>(la, lb, M, N, K, ep, splits, s);
  } else if (ak && !bk) {
    LdKMajor<BM> la{A, lda, M, K}; LdMNMajor<BN> lb{B, ldb, N, K};
    launch_igemm<BM, BN, NPF>(la, lb, M, N, K, ep, splits, s);
  } else if (!ak && bk) {
    LdMNMajor<BM> la{A, lda, M, K}; LdKMajor<BN> lb{B, ldb, N, K};
    launch_igemm<BM, BN, NPF>(la, lb, M, N, K, ep, splits, s);
  } else {
    LdMNMajor<BM> la{A, lda, M, K}; LdMNMajor<BN> lb{B, ldb, N, K};
    launch_igemm<BM, BN, NPF>(la, lb, M, N, K, ep, splits, s);
  }
}

template <int BM, int BN>
static void gemm_tile(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk,
                      int M, int N, int K, Epi ep, int splits, hipStream_t s) {
  // register prefetch depth 1: depths 2 / 3 (igemm_kernel NPF) measured equal
  // on the Transformer / GNMT igemm shapes (profiles/r3/s3/ab_igemm_prefetch_depth.json)
  gemm_tile_p<BM, BN, 1>(A, lda, ak, B, ldb, bk, M, N, K, ep, splits, s);
}

// tuning hook: force tile config / split count (-1 = heuristic); used by
// tools/sweep_gemm.py to measure the policy, never set in training
static int g_force_cfg = -1, g_force_splits = -1;
TAM_KNOB(g_force_cfg) TAM_KNOB(g_force_splits)
void gemm_force(int cfg, int splits) { g_force_cfg = cfg; g_force_splits = splits; }
// LDS-DMA pipelined GEMM (gemm_dma.h) for plain gemm() calls: policy 1 = on
// where eligible, 0 = off (default: measured slower than the igemm on most
// zoo shapes, profiles/gemm_budget_r1.json — the op binding routes per shape
// by measurement instead, gemm_select(path=2)); cfg >= 0 forces its tile
// config (tests / sweeps)
static int g_dma = 0, g_dma_cfg = -1;
TAM_KNOB(g_dma) TAM_KNOB(g_dma_cfg)
void gemm_dma_policy(int policy, int cfg) { g_dma = policy; g_dma_cfg = cfg; }

__global__ void __launch_bounds__(256) zero_kernel(uint4* __restrict__ p16, long n16,
                                                   unsigned char* __restrict__ tail, int ntail) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    p16[i] = make_uint4(0u, 0u, 0u, 0u);
  if (blockIdx.x == 0 && (int)threadIdx.x < ntail) tail[threadIdx.x] = 0;
}

__global__ void __launch_bounds__(256) zero2d_kernel(float* __restrict__ p, long ld, int cols,
                                                     long total) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride)
    p[(i / cols) * ld + i % cols] = 0.f;
}

void zero_async_2d(float* p, long ld, int cols, int rows, hipStream_t s) {
  const long total = (long)cols * rows;
  if (total <= 0) return;
  long blocks = (total + 255) / 256;
  blocks = blocks > 4096 ? 4096 : blocks;
  hipLaunchKernelGGL(zero2d_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, ld, cols, total);
}

void zero_async(void* p, size_t bytes, hipStream_t s) {
  if (bytes == 0) return;
  unsigned char* b = (unsigned char*)p;
  // unaligned head (never hit by torch allocations) handled as a tail launch
  const size_t head = (16 - ((uintptr_t)b & 15)) & 15;
  if (head) {
    const int h = (int)(head < bytes ? head : bytes);
    hipLaunchKernelGGL(zero_kernel, dim3(1), dim3(256), 0, s, (uint4*)nullptr, 0L, b, h);
    b += h;
    bytes -= h;
    if (!bytes) return;
  }
  const long n16 = (long)(bytes / 16);
  int ntail = (int)(bytes % 16);
  long blocks = (n16 + 255) / 256;
  blocks = blocks < 1 ? 1 : blocks > 4096 ? 4096 : blocks;
  hipLaunchKernelGGL(zero_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (uint4*)b, n16,
                     b + n16 * 16, ntail);
}

// LDS-DMA all-layout kernels (gemm8p.h): 0 off (legacy kernels only),
// 1 auto (big GEMMs of every layout), 2 forced wherever eligible, 3 forced
// with slab split-K (the op binding; tests / sweeps). tile: 0 auto,
// 128 / 256 forced (tests / sweeps)
static int g_p8 = 1, g_p8_tile = 0, g_p8_group = 4;
TAM_KNOB(g_p8) TAM_KNOB(g_p8_tile) TAM_KNOB(g_p8_group)
int gemm8p_policy_mode() { return g_p8; }
int gemm8p_policy_tile() { return g_p8_tile; }
void gemm8p_group(int g) { g_p8_group = g > 0 ? g : 4; }
void gemm8p_policy(int mode, int tile) {
  g_p8 = mode;
  g_p8_tile = tile == 64 || tile == 65 || tile == 128 || tile == 129 || tile == 256 ? tile : 0;
}

// block shape of a tile code (64 = 64 x 128; 65 = 64 x 128 with the block's
// K range split over two wave groups, gemm8p_ks2_kernel; 129 = 128 x 128 so)
static int p8_bm(int T) { return T == 65 ? 64 : T == 129 ? 128 : T; }
static int p8_bn(int T) { return T == 256 ? 256 : 128; }
static long p8_tiles(int M, int N, int T) { return (long)cdiv(M, p8_bm(T)) * cdiv(N, p8_bn(T)); }
// blocks that fill the chip: 256^2 one per CU (200 of 256 is enough), 128^2
// two per CU, 64x128 one per CU (the tile exists for ~256-block grids)
static long p8_want(int T) { return T == 128 ? 448 : T == 256 ? 200 : 256; }
static bool p8_known(int T) { return T == 64 || T == 65 || T == 128 || T == 129 || T == 256; }

TAM_P8_VARIANTS(TAM_P8_EXTERN)
TAM_P8_KS2_VARIANTS(TAM_P8_KS2_EXTERN)

template <int BM, int BN, int WNW>
static void p8_launch_l(bool ak, bool bk, const P8Args& g, const Epi& ep, dim3 grid, hipStream_t s) {
  if (ak && bk) p8_launch_one<BM, BN, WNW, true, true>(g, ep, grid, s);
  else if (ak) p8_launch_one<BM, BN, WNW, true, false>(g, ep, grid, s);
  else if (bk) p8_launch_one<BM, BN, WNW, false, true>(g, ep, grid, s);
  else p8_launch_one<BM, BN, WNW, false, false>(g, ep, grid, s);
}

int gemm8p_tile(int M, int N, int K) {
  if (g_p8_tile) return g_p8_tile;   // (a forced 64 falls back to 128 for M-major A: gemm8p_tile_ok)
  // 256^2 only when its grid already covers the chip
  const long t256 = (long)cdiv(M, 256) * cdiv(N, 256);
  return t256 >= 200 ? 256 : 128;
}

void launch_gemm8p(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk, int M,
                   int N, int K, const Epi& ep, int splits, hipStream_t s, int tile) {
  int T = p8_known(tile) ? tile : 256;
  if (!gemm8p_tile_ok(T, ak)) T = 128;
  const int ktiles = K / P8_BK;
  // the two K groups of tile 65 must meet the same barriers: one slice, an
  // even K-tile count (else the plain 64 x 128 tile)
  if (T == 65 && (splits > 1 || ktiles % 2 != 0)) T = 64;
  if (T == 129 && (splits > 1 || ktiles % 2 != 0)) T = 128;
  const int tiles = (int)p8_tiles(M, N, T);
  const int kps = cdiv(ktiles, splits < 1 ? 1 : splits);
  const int z = cdiv(ktiles, kps);
  P8Args g{A, lda, B, ldb, M, N, K, kps, g_p8_group};
  const dim3 grid(tiles, 1, z);
  if (T == 65) {
    if (bk) p8_launch_ks2<64, 128, 2, true, true>(g, ep, grid, s);
    else p8_launch_ks2<64, 128, 2, true, false>(g, ep, grid, s);
  } else if (T == 129) {
    if (bk) p8_launch_ks2<128, 128, 2, true, true>(g, ep, grid, s);
    else p8_launch_ks2<128, 128, 2, true, false>(g, ep, grid, s);
  } else if (T == 64) {
    if (bk) p8_launch_one<64, 128, 2, true, true>(g, ep, grid, s);
    else p8_launch_one<64, 128, 2, true, false>(g, ep, grid, s);
  } else if (T == 128) {
    p8_launch_l<128, 128, 2>(ak, bk, g, ep, grid, s);
  } else {
    p8_launch_l<256, 256, 4>(ak, bk, g, ep, grid, s);
  }
}

// ---- slab split-K (gemm8p.h): reduce ws[sp][M][N] -> C with the epilogue
__global__ void __launch_bounds__(256) p8_slab_reduce_kernel(const float* __restrict__ ws, int sp,
                                                             int M, int N, Epi ep) {
  const long mn = (long)M * N;
  const long n4 = mn >> 2;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 acc = ((const float4*)ws)[i];
    for (int z = 1; z < sp; ++z) {
      const float4 v = ((const float4*)(ws + z * mn))[i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    float vv[4] = {acc.x, acc.y, acc.z, acc.w};
    const long e0 = i << 2;
    const int row = (int)(e0 / N), col0 = (int)(e0 % N);   // N % 4 == 0: one row per float4
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int col = col0 + e;
      float v = vv[e] * ep.alpha + (ep.bias ? bf2f(ep.bias[col]) : 0.f);
      if (ep.relu) v = fmaxf(v, 0.f);
      if (ep.mask && bf2f(ep.mask[(long)row * ep.ldm + col]) <= 0.f) v = 0.f;
      const long off = (long)row * ep.ldc + col;
      if (ep.c_f32) {
        float* c = (float*)ep.c;
        c[off] = ep.mode == 1 ? c[off] + v : v;
      } else {
        bf16_t* c = (bf16_t*)ep.c;
        c[off] = f2bf(ep.mode == 1 ? v + bf2f(c[off]) : v);
      }
    }
  }
}

static int g_p8_force_sp = 0;   // > 0: slab split count forced (A/B sweeps)
TAM_KNOB(g_p8_force_sp)
void gemm8p_slab_force(int sp) { g_p8_force_sp = sp > 0 ? sp : 0; }

int gemm8p_slab_splits(int M, int N, int K, int tile) {
  if (g_p8_force_sp) return g_p8_force_sp;
  const int T = p8_known(tile) ? tile : 256;
  const long t = p8_tiles(M, N, T);
  const int kt = K / P8_BK;
  const long want = p8_want(T);
  if (t >= want * 3 / 4 || kt < 16 || N % 4 != 0) return 1;
  int sp = (int)((want + t - 1) / t);
  if (sp > kt / 8) sp = kt / 8;          // >= 8 K-tiles per slice
  if (sp > 16) sp = 16;
  return sp < 2 ? 1 : sp;
}

void gemm8p_splitk(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk, int M,
                   int N, int K, const Epi& ep, int splits, float* ws, hipStream_t s, int tile) {
  Epi se;
  se.c = ws;
  se.ldc = N;
  se.c_f32 = 1;
  se.mode = 3;
  se.zstride = (long)M * N;
  launch_gemm8p(A, lda, ak, B, ldb, bk, M, N, K, se, splits, s, tile);
  const int ktiles = K / P8_BK;
  const int z = cdiv(ktiles, cdiv(ktiles, splits));   // slabs actually written
  gemm_slab_reduce(ws, z, M, N, ep, s);
}

void gemm_slab_reduce(const float* ws, int sp, int M, int N, const Epi& ep, hipStream_t s) {
  const long n4 = (long)M * N / 4;
  long blocks = (n4 + 255) / 256;
  blocks = blocks > 2048 ? 2048 : blocks;
  hipLaunchKernelGGL(p8_slab_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ws, sp, M, N, ep);
}

// atomic split-K count (fp32 outputs) that fills the chip (>= 4 K-tiles per split)
static int p8_splits(int M, int N, int K, bool can_split, int tile) {
  const long t = p8_tiles(M, N, tile);
  const long want = p8_want(tile);
  if (!can_split || t >= want || K / P8_BK < 8) return 1;
  int sp = (int)((want + t - 1) / t);
  if (sp > K / P8_BK / 4) sp = K / P8_BK / 4;
  return sp < 1 ? 1 : sp;
}

// the register-staged igemm with the heuristic tile, never split -- the
// route gemm_select takes for shallow-K shapes; its bf16 epilogue honours
// Epi::stats (BatchNorm sums of a pointwise conv's output)
void gemm_igemm(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk, int M, int N,
                int K, const Epi& ep, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  TileChoice t = choose_tiles_gemm(M, N, K, false);
  switch (t.cfg > 3 ? 0 : t.cfg) {
    case 0: gemm_tile<128, 128>(A, lda, ak, B, ldb, bk, M, N, K, ep, 1, s); break;
    case 1: gemm_tile<128, 64>(A, lda, ak, B, ldb, bk, M, N, K, ep, 1, s); break;
    case 2: gemm_tile<64, 128>(A, lda, ak, B, ldb, bk, M, N, K, ep, 1, s); break;
    default: gemm_tile<64, 64>(A, lda, ak, B, ldb, bk, M, N, K, ep, 1, s); break;
  }
}

void gemm(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk, int M, int N,
          int K, Epi ep, bool allow_split, hipStream_t s) {
  gemm_select(A, lda, ak, B, ldb, bk, M, N, K, ep, allow_split, s, g_dma ? 2 : 0);
}

// would gemm_select's own size rule put this shape on the 256^2/128^2
// LDS-DMA kernel (path 0 / 1 calls)? The bias-gradient fusion (colsum_a, an
// igemm-only epilogue) is then not worth the igemm fallback
bool gemm_select_big_p8(bool ak, bool bk, int M, int N, int K, long lda, long ldb) {
  if (!(g_p8 > 0 && g_force_cfg < 0 && gemm8p_ok(ak, bk, M, N, K, lda, ldb))) return false;
  const long t8 = (long)cdiv(M, 256) * cdiv(N, 256);
  const double flop = 2.0 * M * N * K;
  return g_p8 >= 2 || (t8 >= 48 && K >= 512 && flop >= 4e9);
}

void gemm_select(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk, int M,
                 int N, int K, Epi ep, bool allow_split, hipStream_t s, int path) {
  if (M <= 0 || N <= 0) return;
  const bool can_split = allow_split && ep.c_f32 && !ep.relu && !ep.mask;
  // (Epi::colsum_a is an igemm-only epilogue: no LDS-DMA kernels then)
  if (g_p8 > 0 && g_force_cfg < 0 && !ep.colsum_a && gemm8p_ok(ak, bk, M, N, K, lda, ldb)) {
    const long t8 = (long)cdiv(M, 256) * cdiv(N, 256);
    const double flop = 2.0 * M * N * K;
    if (g_p8 >= 2 || path == 3 || (t8 >= 48 && K >= 512 && flop >= 4e9)) {
      int tile = gemm8p_tile(M, N, K);
      if (!gemm8p_tile_ok(tile, ak)) tile = 128;
      int sp = p8_splits(M, N, K, can_split, tile);
      if (g_force_splits >= 1) sp = can_split ? g_force_splits : 1;
      prepare_split(ep, sp, M, N, s);
      launch_gemm8p(A, lda, ak, B, ldb, bk, M, N, K, ep, sp, s, tile);
      return;
    }
  }
  TileChoice t = choose_tiles_gemm(M, N, K, can_split);
  if (g_force_cfg >= 0) t.cfg = g_force_cfg;
  if (g_force_splits >= 1) t.splits = can_split ? g_force_splits : 1;
  // 256x256 LDS-DMA kernel for large K-major x K-major problems
  const long t256 = (long)cdiv(M, 256) * cdiv(N, 256);
  const bool big = !ep.colsum_a && gemm256_ok(ak, bk, M, N, K, lda, ldb) &&
                   (t.cfg == 4 || (g_force_cfg < 0 && t256 >= 192 && K >= 1024));
  if (!big && path == 2 && g_force_cfg < 0 && !ep.colsum_a && gemm_dma_ok(A, lda, ak, B, ldb, bk, M, N, K, ep)) {
    GdChoice c = gemm_dma_choose(M, N, K, can_split);
    if (g_dma_cfg >= 0) c.cfg = g_dma_cfg;
    if (g_force_splits >= 1) c.splits = can_split ? g_force_splits : 1;
    prepare_split(ep, c.splits, M, N, s);
    launch_gemm_dma(A, lda, ak, B, ldb, bk, M, N, K, ep, c.cfg, c.splits, s);
    return;
  }
  if (big) {
    int sp = 1;
    if (g_force_splits >= 1) sp = t.splits;
    else if (can_split && t256 < 256 && K / 64 >= 8) {
      sp = (int)((256 + t256 - 1) / t256);
      if (sp > K / 64 / 4) sp = K / 64 / 4;
      if (sp < 1) sp = 1;
    }
    prepare_split(ep, sp, M, N, s);
    launch_gemm256(A, lda, B, ldb, M, N, K, ep, sp, s);
    return;
  }
  if (t.cfg > 3) t.cfg = 0;
  prepare_split(ep, t.splits, M, N, s);
  switch (t.cfg) {
    case 0: gemm_tile<128, 128>(A, lda, ak, B, ldb, bk, M, N, K, ep, t.splits, s); break;
    case 1: gemm_tile<128, 64>(A, lda, ak, B, ldb, bk, M, N, K, ep, t.splits, s); break;
    case 2: gemm_tile<64, 128>(A, lda, ak, B, ldb, bk, M, N, K, ep, t.splits, s); break;
    default: gemm_tile<64, 64>(A, lda, ak, B, ldb, bk, M, N, K, ep, t.splits, s); break;
  }
}

}  // namespace tam
