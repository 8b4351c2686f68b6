// tiresias_amd — MFMA GEMM entry points (all four operand majorities) and the
// tile / split-K selection heuristic shared with the conv passes.
#include "tam/launch.h"
#include "tam/tiles.h"

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

void gemm(const bf16_t* A, long lda, bool ak, const bf16_t* B, long ldb, bool bk, int M, int N,
          int K, Epi ep, bool allow_split, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  TileChoice t = choose_tiles(M, N, K, allow_split && ep.c_f32 && !ep.relu && !ep.mask);
  prepare_split(ep, t.splits, M, N, s);
  switch (t.cfg) {
    case 0: gemm_tile<128, 128>(A, lda, ak, B, ldb, bk, M, N, K, ep, t.splits, s); break;
    case 1: gemm_tile<128, 64>(A, lda, ak, B, ldb, bk, M, N, K, ep, t.splits, s); break;
    case 2: gemm_tile<64, 128>(A, lda, ak, B, ldb, bk, M, N, K, ep, t.splits, s); break;
    default: gemm_tile<64, 64>(A, lda, ak, B, ldb, bk, M, N, K, ep, t.splits, s); break;
  }
}

}  // namespace tam
