// tiresias_amd — 256x256 LDS-DMA MFMA GEMM with FOUR waves (one per SIMD),
// each owning a 128x128 output block: C[M][N] = A[M][K] . B[N][K]^T, both
// operands K-major, bf16 out.
//
// Why next to gemm8p (8 waves of 128x64): per K-tile of 64 a CU's waves read
// (rows + cols) x 64 x 2 B of fragments from LDS each. 8 waves of 128x64 read
// 8 x 24 KB = 192 KB per 8.4 MFLOP; 4 waves of 128x128 read 4 x 32 KB =
// 128 KB for the same work (MI355X_MICROARCH.md §LDS: ds_read_b128 at
// 256 B/clk/CU), so the LDS array is busy 1/3 less per MFMA cycle. The price:
// 256 fp32 accumulators per lane (AGPR/VGPR file of 512 at one wave per SIMD)
// and no second wave on the SIMD to hide LDS latency -- fragments of the next
// k-step are requested before the current MFMA cluster.
//
// Pipeline: 2 LDS stages of 64 KB; per K-tile ONE counted wait (vmcnt 0 on
// this thread's DMAs of tile t, issued a whole K-tile earlier) and ONE barrier,
// then tile t+1's 16 DMA instructions per thread go out and tile t is computed
// (2 k-steps x 64 MFMAs per wave). K-major image and swizzle as gemm8p
// (kmaj_off: 16-B chunk c of row r at c ^ ((r>>1)&7), applied on the SOURCE).
//
// Measured (tools/ab_gemm4w.py, profiles/r2/gemm4w_ab.json, interleaved in one
// process): 4096^3 median 1043 TF/s (PIPE 1) vs gemm8p 1204; 8192^3 1154 vs
// 1323. One wave per SIMD leaves the barrier / first-fragment latency of every
// K-tile exposed, which costs more than the LDS traffic saved; not routed --
// kept as the measured alternative and a numerics-tested kernel.
#pragma once
#include "tam/igemm.h"

namespace tam {

typedef __attribute__((address_space(3))) void g4_lds_t;

// PIPE 0: per k-step, read its 16 fragments then run its 64 MFMAs; PIPE 1:
// all 32 fragments of the K-tile requested up front (128 VGPRs), so the
// second k-step's reads land under the first k-step's MFMA cluster
template <int PIPE>
__global__ void __launch_bounds__(256, 1) gemm4w_kernel(const bf16_t* __restrict__ A, long lda,
                                                        const bf16_t* __restrict__ B, long ldb,
                                                        bf16_t* __restrict__ C, long ldc, int M, int N,
                                                        int K, int group) {
  constexpr int BM = 256, BN = 256, BK = 64;
  constexpr int TILE = BM * BK * 2;            // 32 KB per operand per stage
  constexpr int STAGE = 2 * TILE;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid & 1, wn = wid >> 1;

  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = group * tiles_n;
  const int grp = bid / per_group;
  const int first_m = grp * group;
  const int gsize = min(tiles_m - first_m, group);
  const int tm = first_m + (bid % per_group) % gsize;
  const int tn = (bid % per_group) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = K / BK;

  // DMA: one wave-instruction fills one 1-KiB group = 8 rows x 128 B; group
  // g = 4 j + wid, row r = 8 g + lane/8, source chunk (lane%8) ^ ((r>>1)&7)
  // (independent of j: (32 j >> 1) & 7 == 0)
  const int r_lane = wid * 8 + (lane >> 3);
  const int csrc = ((lane & 7) ^ ((r_lane >> 1) & 7)) * 8;
  auto issue = [&](int t, int st) {
    char* sa = smem + st * STAGE;
    char* sb = sa + TILE;
    const int k0 = t * BK + csrc;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = r_lane + 32 * j;
      const int ra = min(m0 + r, M - 1), rb = min(n0 + r, N - 1);   // edge rows are never stored
      __builtin_amdgcn_global_load_lds((const void*)(A + (long)ra * lda + k0),
                                       (g4_lds_t*)(sa + (4 * j + wid) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(B + (long)rb * ldb + k0),
                                       (g4_lds_t*)(sb + (4 * j + wid) * 1024), 16, 0, 0);
    }
  };

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) issue(0, 0);
  for (int t = 0; t < nk; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();              // tile t landed everywhere; tile t-1 reads retired
    asm volatile("" ::: "memory");
    if (t + 1 < nk) issue(t + 1, (t + 1) & 1);
    const char* sa = smem + (t & 1) * STAGE;
    const char* sb = sa + TILE;
    if constexpr (PIPE == 0) {
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        s16x8_t fa[8], fb[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) fb[j] = read_frag_k(sb, lane, wn * 128 + 16 * j, kk);
#pragma unroll
        for (int i = 0; i < 8; ++i) fa[i] = read_frag_k(sa, lane, wm * 128 + 16 * i, kk);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[i]),
                                                                __builtin_bit_cast(bf16x8_t, fb[j]),
                                                                acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    } else {
      s16x8_t fa[2][8], fb[2][8];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int j = 0; j < 8; ++j) fb[kk][j] = read_frag_k(sb, lane, wn * 128 + 16 * j, kk);
#pragma unroll
        for (int i = 0; i < 8; ++i) fa[kk][i] = read_frag_k(sa, lane, wm * 128 + 16 * i, kk);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        // in-order LDS returns: k-step 0 needs the first 16 of 32 reads
        // (lgkmcnt counts to 15 at most: waits for 17)
        if (kk == 0) asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[kk][i]),
                                                                __builtin_bit_cast(bf16x8_t, fb[kk][j]),
                                                                acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  __syncthreads();                               // stages free: epilogue slabs

  // LDS-staged bf16 epilogue: 32 rows x 128 columns per wave per pass,
  // written back as 16-B row chunks. C/D map of 16x16x32: col = lane & 15,
  // row = 4 (lane >> 4) + r
  constexpr int LDW = 128 + 8;
  bf16_t* slab = (bf16_t*)(smem + wid * (32 * LDW * 2));
#pragma unroll
  for (int h = 0; h < 4; ++h) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          slab[(16 * ii + 4 * (lane >> 4) + r) * LDW + 16 * j + (lane & 15)] = f2bf(acc[2 * h + ii][j][r]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = u * 64 + lane, lr = idx >> 4, ch = idx & 15;
      const int row = m0 + wm * 128 + 32 * h + lr, col = n0 + wn * 128 + ch * 8;
      if (row < M && col + 8 <= N)
        *(uint4*)(C + (long)row * ldc + col) = *(const uint4*)(slab + lr * LDW + ch * 8);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

inline bool gemm4w_ok(int M, int N, int K, long lda, long ldb, long ldc) {
  return K % 64 == 0 && K >= 64 && M >= 1 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0;
}

inline void launch_gemm4w(const bf16_t* A, long lda, const bf16_t* B, long ldb, bf16_t* C, long ldc, int M,
                          int N, int K, int group, int pipe, hipStream_t s) {
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  if (pipe)
    hipLaunchKernelGGL(gemm4w_kernel<1>, dim3(tiles), dim3(256), 0, s, A, lda, B, ldb, C, ldc, M, N, K,
                       group > 0 ? group : 4);
  else
    hipLaunchKernelGGL(gemm4w_kernel<0>, dim3(tiles), dim3(256), 0, s, A, lda, B, ldb, C, ldc, M, N, K,
                       group > 0 ? group : 4);
}

}  // namespace tam
