// tiresias_amd — host-side launch API of the HIP kernel library.
// Plain C++ over raw device pointers + hipStream_t; the torch binding layer
// (csrc/bindings/ops.cpp) is the only TU that sees ATen.
#pragma once
#include <hip/hip_runtime.h>
#include "tam/igemm.h"

namespace tam {

// C[M,N] (op)= alpha * A(m,k) B(k,n) (+bias)(relu)(mask)
//   A(m,k) = a_kmajor ? A[m*lda+k] : A[k*lda+m]
//   B(k,n) = b_kmajor ? B[n*ldb+k] : B[k*ldb+n]
// allow_split: permit split-K (fp32 atomic output; C is zeroed first when
// ep.mode == 0, requires ldc == N).
// the heuristic-tile igemm, unsplit (Epi::stats honoured in its bf16 epilogue)
void gemm_igemm(const bf16_t* A, long lda, bool a_kmajor, const bf16_t* B, long ldb, bool b_kmajor, int M,
                int N, int K, const Epi& ep, hipStream_t s);
void gemm(const bf16_t* A, long lda, bool a_kmajor, const bf16_t* B, long ldb, bool b_kmajor,
          int M, int N, int K, Epi ep, bool allow_split, hipStream_t s);
// path 0: heuristic, 2: LDS-DMA GEMM where eligible, 3: gemm8p where eligible
void gemm_select(const bf16_t* A, long lda, bool a_kmajor, const bf16_t* B, long ldb, bool b_kmajor,
                 int M, int N, int K, Epi ep, bool allow_split, hipStream_t s, int path);
void gemm_force(int cfg, int splits);   // tuning hook (-1 = heuristic)
void gemm_dma_policy(int policy, int cfg);   // LDS-DMA GEMM on/off, forced tile cfg (-1 auto)
// 256^2 all-layout LDS-DMA GEMM: 0 off, 1 auto (big GEMMs), 2 forced where eligible
void gemm8p_policy(int mode, int tile);   // tile 128 / 256: forced (tests), else auto
// pointwise-conv GEMM (gemm_pw.hip): C[M][N] = A[M][K] . B[N][K]^T for many
// pixels (M >= 65536), K, N in {64, 128, 256}, K * N <= 16384; ReLU-backward
// mask / BN statistics (fp64 [BN_SHARDS][2N]) / relu as in Epi. false: not
// eligible, nothing launched
bool gemm_pw(const bf16_t* A, long lda, const bf16_t* B, long ldb, bf16_t* C, long ldc, long M, int N, int K,
             const bf16_t* mask, long ldm, double* stats, int relu, hipStream_t s);
bool gemm_pw_ok(long M, int N, int K, long lda, long ldb, long ldc);
void gemm_pw_policy(int on);   // 0: pointwise convs on the dense GEMM route (A/B)
void gemm8p_group(int g);   // M-tiles per tile-order group of gemm8p (default 4)
int gemm8p_policy_mode();

// Grouped weight-gradient GEMM (gemm_grouped.hip): for every problem p,
//   C_p[M][N] (+)= A_p^T B_p  (A_p [K][lda] M-major, B_p [K][ldb] N-major, fp32 C row stride N)
//   bias_p[M] += column sums of A_p (when bias_p != null)
// in ONE launch per P8G_MAX problems (gemm8p 128^2 tiles + column-sum blocks).
struct GGProblem {
  const bf16_t* A;
  const bf16_t* B;
  float* C;
  float* bias;
  int M, N, K, lda, ldb;
  int mode = 1;      // 0: C = A^T B (store), 1: C += A^T B
};
void gemm_wgrad_grouped(const GGProblem* probs, int n, hipStream_t s);
// deferred conv weight-gradient slab reduces, one launch per 40:
// dw[e] = (mode[e] ? dw[e] : 0) + sum_z ws[e][z][:mn[e]]
void wgrad_slab_reduce_many(const float* const* ws, const int* sp, const long* mn, float* const* dw,
                            const int* mode, int n, hipStream_t s);
bool gemm_wgrad_grouped_ok(int M, int N, int K, long lda, long ldb);
void gemm_grouped_tile(int t);   // 128 (default) or 256

// split-K slab reduce: C (op)= epilogue(sum_z ws[z][M][N]) -- N % 4 == 0
void gemm_slab_reduce(const float* ws, int sp, int M, int N, const Epi& ep, hipStream_t s);

// Skinny-M weight-streaming GEMM (gemm_skinny.hip): A K-major [M][K] with
// M <= 64, B K-major or N-major, K % 64 == 0. sp K-slices (gemm_skinny_splits);
// sp > 1 needs ws = fp32 [sp][M][N] and N % 4 == 0.
bool gemm_skinny_ok(bool ak, bool bk, int M, int N, int K, long lda, long ldb);
int gemm_skinny_splits(int M, int N, int K);
void gemm_skinny(const bf16_t* A, long lda, const bf16_t* B, long ldb, bool bk, int M, int N, int K,
                 const Epi& ep, int sp, float* ws, hipStream_t s);
// on: 0 off / 1 on; force_splits > 0 forces the K-slice count; nst: LDS ring depth 3 or 4
void gemm_skinny_policy(int on, int force_splits, int nst);

// NHWC convolutions, weights [K][R][S][C] (C, K multiples of 8)
// ws / ws_floats: split-K scratch of conv_*_split_ws(g) floats (none: unsplit)
int conv_fwd(const bf16_t* x, const bf16_t* w, const ConvGeom& g, Epi ep, hipStream_t s, float* ws = nullptr,
             long ws_floats = 0);
long conv_fwd_split_ws(const ConvGeom& g);
// ResNet stem (7x7 / s2 / p3, C 8 -> K 64) forward kernel; false: not its shape
bool conv_stem_fwd(const bf16_t* x, const bf16_t* w, const ConvGeom& g, const Epi& ep, hipStream_t s);
void conv_stem_policy(int p);   // 1: stem kernels where they apply (default), 0: generic paths
// stem weight gradient (per-CU fp32 partial slabs + reduce); ws: conv_stem_wgrad_ws(g) floats
long conv_stem_wgrad_ws(const ConvGeom& g);
bool conv_stem_wgrad(const bf16_t* dy, const bf16_t* x, const ConvGeom& g, float* dw, int mode, float* ws,
                     long ws_floats, hipStream_t s);
long conv_dgrad_split_ws(const ConvGeom& g);
void conv_split_policy(int p);   // 1: split-K of under-filled LDS-DMA passes (default), 0: off
// dx[N*H*W][C]; wt = conv_weight_t(w) laid out [C][R][S][K] (ignored for 1x1/s1)
int conv_dgrad(const bf16_t* dy, const bf16_t* w, const bf16_t* wt, const ConvGeom& g, Epi ep,
               hipStream_t s, float* ws = nullptr, long ws_floats = 0);
// dw[K][R*S*C] fp32, ep.mode 0 (overwrite) or 1 (accumulate)
// ws / ws_floats: slab split-K scratch of conv_wgrad_split_ws(g) floats (none: atomics)
int conv_wgrad(const bf16_t* dy, const bf16_t* x, const ConvGeom& g, Epi ep, hipStream_t s,
               float* dbias = nullptr, bool allow_patch = true, float* ws = nullptr, long ws_floats = 0,
               int* slab_defer = nullptr);
long conv_wgrad_split_ws(const ConvGeom& g);
void conv_wgrad_slab_policy(int p);   // 1: slab split-K for the DMA wgrad (default), 0: fp32 atomics
void conv_weight_t(const bf16_t* w, bf16_t* wt, const ConvGeom& g, hipStream_t s);
void conv_dma_policy(int p);   // 1: LDS-DMA core where eligible (default), 0: igemm only
// LDS-DMA wgrad tile / split (0: heuristic); noatomic: timing-only racy adds
void conv_wgrad_force(int bm, int bn, int splits, int noatomic = 0);
void conv_wgrad_order(int flat);    // DMA wgrad block order: 1 split-major XCD remap (default), 0 3-D grid
void conv_wgrad_c64_policy(int p);   // 64-channel 3x3 wgrad kernel: 1 on (default), 0 off, >= 2 blocks per k-slice
void conv_halo_policy(int p);   // 1: 64-channel 3x3 stride-1 passes on the halo-tile kernel (default)
bool gemm_select_big_p8(bool ak, bool bk, int M, int N, int K, long lda, long ldb);   // plain-GEMM igemm K-tiles in flight (1..3)

}  // namespace tam
