// tiresias_amd — MFMA GEMM entry points (all four operand majorities) and the
// tile / split-K selection heuristic shared with the conv passes.
#include "tam/launch.h"
#include "tam/tiles.h"
#include "tam/gemm256.h"

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

void gemm(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk, int M, int N,
          int K, Epi ep, bool allow_split, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  const bool can_split = allow_split && ep.c_f32 && !ep.relu && !ep.mask;
  TileChoice t = choose_tiles_gemm(M, N, K, can_split);
  if (g_force_cfg >= 0) t.cfg = g_force_cfg;
  if (g_force_splits >= 1) t.splits = can_split ? g_force_splits : 1;
  // 256x256 LDS-DMA kernel for large K-major x K-major problems
  const long t256 = (long)cdiv(M, 256) * cdiv(N, 256);
  const bool big = gemm256_ok(ak, bk, M, N, K, lda, ldb) &&
                   (t.cfg == 4 || (g_force_cfg < 0 && t256 >= 192 && K >= 1024));
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
