// tiresias_amd — tile-shape / split-K selection and the typed launcher for the
// implicit-GEMM core. Sized for 256 CUs: prefer the largest tile that still
// yields >= 256 workgroups, otherwise shrink tiles, then split K (fp32 atomics).
#pragma once
#include "tam/igemm.h"

namespace tam {

struct TileChoice { int cfg; int splits; };   // cfg: 0=128x128 1=128x64 2=64x128 3=64x64

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

inline TileChoice choose_tiles(int M, int N, int K, bool can_split) {
  static const int bm[4] = {128, 128, 64, 64}, bn[4] = {128, 64, 128, 64};
  int best = 3;
  for (int c = 0; c < 4; ++c) {
    if (M <= 64 && bm[c] == 128) continue;
    if (N <= 64 && bn[c] == 128) continue;
    const long tiles = (long)cdiv(M, bm[c]) * cdiv(N, bn[c]);
    if (tiles >= 256) { best = c; break; }
  }
  TileChoice t{best, 1};
  if (can_split) {
    const long tiles = (long)cdiv(M, bm[best]) * cdiv(N, bn[best]);
    const int ktiles = cdiv(K, IG_BK);
    if (tiles < 512 && ktiles >= 8) {
      int sp = (int)((512 + tiles - 1) / tiles);
      sp = sp < ktiles / 4 ? sp : ktiles / 4;
      if (sp > 256) sp = 256;   // tiny-output reductions (first-layer wgrad: 64x72) need many
      t.splits = sp < 1 ? 1 : sp;
    }
  }
  return t;
}

// Plain-GEMM policy, fitted to tools/sweep_gemm.py over the zoo's linear
// shapes on MI355X (profiles/sweep_gemm_r1.json; within 0.3% of the per-shape
// best vs 9.8% for choose_tiles): 128x128 only when K is deep enough to
// amortise its prologue/epilogue AND there are >=1 tile per CU; otherwise
// 64x64 (4x the workgroups, better latency hiding); split-K to ~512 WGs.
inline TileChoice choose_tiles_gemm(int M, int N, int K, bool can_split) {
  const long t128 = (long)cdiv(M, 128) * cdiv(N, 128);
  const bool big = M > 64 && N > 64 &&
                   ((K >= 2048 && t128 >= 256) || (K >= 1024 && t128 >= 1024));
  TileChoice t{big ? 0 : 3, 1};
  if (can_split) {
    const int b = big ? 128 : 64;
    const long tiles = (long)cdiv(M, b) * cdiv(N, b);
    const int ktiles = cdiv(K, IG_BK);
    if (tiles < 512 && ktiles >= 8) {
      int sp = (int)((512 + tiles - 1) / tiles);
      if (sp > ktiles / 4) sp = ktiles / 4;
      if (sp > 32) sp = 32;
      t.splits = sp < 1 ? 1 : sp;
    }
  }
  return t;
}

inline void prepare_split(Epi& ep, int splits, int M, int N, hipStream_t s) {
  if (splits <= 1) return;
  if (ep.mode == 0) {
    if (ep.ldc == N) {
      zero_async(ep.c, (size_t)M * N * sizeof(float), s);
    } else {
      zero_async_2d((float*)ep.c, ep.ldc, N, M, s);
    }
  }
  ep.mode = 2;
}

template <int BM, int BN, int NPF = 1, class LA, class LB>
inline void launch_igemm(const LA& la, const LB& lb, int M, int N, int K, const Epi& ep, int splits,
                         hipStream_t s) {
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  const int ktiles = cdiv(K, IG_BK);
  int kps = cdiv(ktiles, splits < 1 ? 1 : splits);
  if (kps < 1) kps = 1;
  const int z = cdiv(ktiles, kps) < 1 ? 1 : cdiv(ktiles, kps);
  dim3 grid(tiles, 1, z);
  hipLaunchKernelGGL((igemm_kernel<BM, BN, LA, LB, NPF>), grid, dim3(IG_THREADS), 0, s, la, lb, M, N, K,
                     kps, ep);
}

}  // namespace tam
