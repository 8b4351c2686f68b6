// tiresias_amd — MFMA GEMM entry points (all four operand majorities) and the
// tile / split-K selection heuristic shared with the conv passes.
#include "tam/launch.h"
#include "tam/tiles.h"
#include "tam/gemm256.h"
#include "tam/gemm_dma.h"

namespace tam {

template <int BM, int BN>
static void gemm_tile(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk,
                      int M, int N, int K, Epi ep, int splits, hipStream_t s) {
  if (ak && bk) {
    LdKMajor<BM> la{A, lda, M, K}; LdKMajor<BN> lb{B, ldb, N, K};
    launch_igemm<BM, BN>(la, lb, M, N, K, ep, splits, s);
  } else if (ak && !bk) {
    LdKMajor<BM> la{A, lda, M, K}; LdMNMajor<BN> lb{B, ldb, N, K};
    launch_igemm<BM, BN>(la, lb, M, N, K, ep, splits, s);
  } else if (!ak && bk) {
    LdMNMajor<BM> la{A, lda, M, K}; LdKMajor<BN> lb{B, ldb, N, K};
    launch_igemm<BM, BN>(la, lb, M, N, K, ep, splits, s);
  } else {
    LdMNMajor<BM> la{A, lda, M, K}; LdMNMajor<BN> lb{B, ldb, N, K};
    launch_igemm<BM, BN>(la, lb, M, N, K, ep, splits, s);
  }
}

// tuning hook: force tile config / split count (-1 = heuristic); used by
// tools/sweep_gemm.py to measure the policy, never set in training
static int g_force_cfg = -1, g_force_splits = -1;
void gemm_force(int cfg, int splits) { g_force_cfg = cfg; g_force_splits = splits; }
// LDS-DMA pipelined GEMM (gemm_dma.h) for plain gemm() calls: policy 1 = on
// where eligible, 0 = off (default: measured slower than the igemm on most
// zoo shapes, profiles/gemm_budget_r1.json — the op binding routes per shape
// by measurement instead, gemm_select(path=2)); cfg >= 0 forces its tile
// config (tests / sweeps)
static int g_dma = 0, g_dma_cfg = -1;
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

void gemm(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk, int M, int N,
          int K, Epi ep, bool allow_split, hipStream_t s) {
  gemm_select(A, lda, ak, B, ldb, bk, M, N, K, ep, allow_split, s, g_dma ? 2 : 0);
}

void gemm_select(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk, int M,
                 int N, int K, Epi ep, bool allow_split, hipStream_t s, int path) {
  if (M <= 0 || N <= 0) return;
  const bool can_split = allow_split && ep.c_f32 && !ep.relu && !ep.mask;
  TileChoice t = choose_tiles_gemm(M, N, K, can_split);
  if (g_force_cfg >= 0) t.cfg = g_force_cfg;
  if (g_force_splits >= 1) t.splits = can_split ? g_force_splits : 1;
  // 256x256 LDS-DMA kernel for large K-major x K-major problems
  const long t256 = (long)cdiv(M, 256) * cdiv(N, 256);
  const bool big = gemm256_ok(ak, bk, M, N, K, lda, ldb) &&
                   (t.cfg == 4 || (g_force_cfg < 0 && t256 >= 192 && K >= 1024));
  if (!big && path == 2 && g_force_cfg < 0 && gemm_dma_ok(A, lda, ak, B, ldb, bk, M, N, K, ep)) {
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
