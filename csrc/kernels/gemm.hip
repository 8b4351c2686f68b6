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
