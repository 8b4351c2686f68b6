// tiresias_amd — 256x256x64 bf16 GEMM for large K-major x K-major problems
// (C[M][N] = A[M][K] . B[N][K]^T, fp32 accumulate, Epi epilogue).
//
// Structure (MI355X-first, see cdna_hip_programming.md §5 "Pipelining across
// barriers" and the 256^2 template discussion):
//  * 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns a 128x64 output
//    block = 8x4 16x16 MFMA tiles (128 fp32 accumulators per lane).
//  * Operands are staged HBM/L2 -> LDS with LDS-DMA (global_load_lds_dwordx4,
//    no VGPR round trip). The LDS image is lane-linear per wave instruction;
//    the XOR bank swizzle (16-B chunk ^ ((row>>1)&7), conflict-free for the
//    16x16x32 ds_read_b128 fragment pattern) is applied on the SOURCE address.
//  * Two LDS stages (2 x 64 KiB), each split into half-tiles by the quadrant
//    that reads them. Per K-tile a wave runs 4 phases = 4 C-quadrants
//    (64 rows x 32 cols x K64 = 16 MFMA):
//        p1 (mh0,nh0) reads A-lo + B-lo     p2 (mh0,nh1) reads B-hi
//        p3 (mh1,nh1) reads A-hi            p4 (mh1,nh0) reads nothing
//    (fragments stay in registers between phases). A half-tile of the stage
//    is refilled with tile t+2 in the phase right after its last reader, so
//    every DMA has >= 5 phases of MFMA work to land; one counted
//    `s_waitcnt vmcnt(8)` per K-tile (only tile t+2's 8 DMAs may remain in
//    flight) followed by the phase barrier retires tile t+1 — the pipeline
//    never drains inside the loop. Raw s_barrier only (no __syncthreads, whose
//    fence would wait vmcnt(0)); all LDS is one __shared__ array.
//  * XCD-aware bijective block remap + grouped-M tile order (L2 reuse).
#pragma once
#include "tam/igemm.h"

namespace tam {

constexpr int G8_BM = 256, G8_BN = 256, G8_BK = 64, G8_THREADS = 512;
constexpr int G8_TILE = G8_BM * G8_BK * 2;   // 32 KiB per operand per stage
constexpr int G8_STAGE = 2 * G8_TILE;

typedef __attribute__((address_space(3))) void lds_void_t;

struct G8Args {
  const bf16_t* A;
  long lda;
  const bf16_t* B;
  long ldb;
  int M, N, K;
  int kps;   // K-tiles per split (blockIdx.z)
};

// Issue one half-tile (128 rows x 64 k = 16 KiB; 2 DMA instructions per
// thread) of a K-major operand. Half h holds the rows whose bit BIT equals h
// (A: bit 6 -> the wave's mh quadrant; B: bit 5 -> the wave's nh quadrant).
// One wave instruction writes one 8-row group (1 KiB, lane-linear).
template <int BIT>
__device__ __forceinline__ void g8_issue_half(const bf16_t* __restrict__ base, long ld, int rows,
                                             int row0, int k0, char* tile, int h, int wid,
                                             int lane) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int g = j * 8 + wid;   // 8-row group 0..15 of this half
    const int r8 = BIT == 6 ? (((g >> 3) << 7) | (h << 6) | ((g & 7) << 3))
                            : (((g >> 2) << 6) | (h << 5) | ((g & 3) << 3));
    const int r = r8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);   // logical 16-B chunk for this LDS slot
    int gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;              // clamp: rows past the edge are never stored
    const bf16_t* src = base + (long)gr * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(tile + r8 * 128), 16, 0, 0);
  }
}

// raw s_barrier fenced for the COMPILER only (keeps LDS reads / DMA issues on
// their side of it); emits no s_waitcnt
__device__ __forceinline__ void g8_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int I0, int J0, int FB>
__device__ __forceinline__ void g8_mfma(f32x4_t (&acc)[8][4], const s16x8_t (&fa)[4][2],
                                        const s16x8_t (&fb)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[I0 + i][J0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(bf16x8_t, fa[i][kk]), __builtin_bit_cast(bf16x8_t, fb[j][kk]),
            acc[I0 + i][J0 + j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}

__global__ void __launch_bounds__(G8_THREADS, 1) gemm256_kernel(G8Args a, Epi ep) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * G8_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;

  const int tiles_m = (a.M + G8_BM - 1) / G8_BM, tiles_n = (a.N + G8_BN - 1) / G8_BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GROUP = 4;
  const int per_group = GROUP * tiles_n;
  const int grp = bid / per_group;
  const int first_m = grp * GROUP;
  const int gsize = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (bid % per_group) % gsize;
  const int tn = (bid % per_group) / gsize;
  const int m0 = tm * G8_BM, n0 = tn * G8_BN;

  const int ktiles = a.K / G8_BK;
  const int kt0 = blockIdx.z * a.kps;
  const int kt1 = min(ktiles, kt0 + a.kps);
  const int nk = kt1 - kt0;

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto issueA = [&](int t, int h) {
    g8_issue_half<6>(a.A, a.lda, a.M, m0, (kt0 + t) * G8_BK, smem + (t & 1) * G8_STAGE, h, wid,
                     lane);
  };
  auto issueB = [&](int t, int h) {
    g8_issue_half<5>(a.B, a.ldb, a.N, n0, (kt0 + t) * G8_BK,
                     smem + (t & 1) * G8_STAGE + G8_TILE, h, wid, lane);
  };

  if (nk > 0) {
    issueA(0, 0); issueB(0, 0); issueB(0, 1); issueA(0, 1);
    if (nk > 1) {
      issueA(1, 0); issueB(1, 0); issueB(1, 1); issueA(1, 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    g8_barrier();

    const int arow = wm * 128, bcol = wn * 64;
    s16x8_t fa[4][2], fb0[2][2], fb1[2][2];
    for (int t = 0; t < nk; ++t) {
      const char* ta = smem + (t & 1) * G8_STAGE;
      const char* tb = ta + G8_TILE;
      const bool pre = t + 2 < nk;
      // ---- p1: quadrant (mh0, nh0)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i][kk] = read_frag_k(ta, lane, arow + 16 * i, kk);
#pragma unroll
        for (int j = 0; j < 2; ++j) fb0[j][kk] = read_frag_k(tb, lane, bcol + 16 * j, kk);
      }
      g8_mfma<0, 0, 0>(acc, fa, fb0);
      g8_barrier();
      // ---- p2: quadrant (mh0, nh1); A-lo / B-lo of this stage are dead -> refill t+2
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < 2; ++j) fb1[j][kk] = read_frag_k(tb, lane, bcol + 32 + 16 * j, kk);
      if (pre) { issueA(t + 2, 0); issueB(t + 2, 0); }
      g8_mfma<0, 2, 1>(acc, fa, fb1);
      g8_barrier();
      // ---- p3: quadrant (mh1, nh1); B-hi dead -> refill
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i][kk] = read_frag_k(ta, lane, arow + 64 + 16 * i, kk);
      if (pre) issueB(t + 2, 1);
      g8_mfma<4, 2, 1>(acc, fa, fb1);
      g8_barrier();
      // ---- p4: quadrant (mh1, nh0); A-hi dead -> refill; retire tile t+1
      if (pre) issueA(t + 2, 1);
      g8_mfma<4, 0, 0>(acc, fa, fb0);
      if (pre) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      g8_barrier();
    }
  }

  // ---- epilogue: C/D map of 16x16x32: col = lane&15, row = (lane>>4)*4 + r
  const bool add_bias = ep.bias != nullptr && blockIdx.z == 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wn * 64 + 16 * j + (lane & 15);
    if (col >= a.N) continue;
    const float bv = add_bias ? bf2f(ep.bias[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 128 + 16 * i + 4 * (lane >> 4) + r;
        if (row >= a.M) continue;
        float v = acc[i][j][r] * ep.alpha + bv;
        if (ep.relu) v = fmaxf(v, 0.f);
        if (ep.mask && bf2f(ep.mask[(long)row * ep.ldm + col]) <= 0.f) v = 0.f;
        const long off = (long)row * ep.ldc + col;
        if (ep.c_f32) {
          float* c = (float*)ep.c;
          if (ep.mode == 2) atomicAdd(c + off, v);
          else if (ep.mode == 1) c[off] += v;
          else c[off] = v;
        } else {
          bf16_t* c = (bf16_t*)ep.c;
          if (ep.mode == 1) v += bf2f(c[off]);
          c[off] = f2bf(v);
        }
      }
    }
  }
}

inline bool gemm256_ok(bool ak, bool bk, int M, int N, int K, long lda, long ldb) {
  return ak && bk && K % G8_BK == 0 && K >= G8_BK && lda % 8 == 0 && ldb % 8 == 0 && M >= 128 &&
         N >= 128;
}

inline void launch_gemm256(const bf16_t* A, long lda, const bf16_t* B, long ldb, int M, int N,
                           int K, const Epi& ep, int splits, hipStream_t s) {
  const int tiles = cdiv(M, G8_BM) * cdiv(N, G8_BN);
  const int ktiles = K / G8_BK;
  int kps = cdiv(ktiles, splits < 1 ? 1 : splits);
  const int z = cdiv(ktiles, kps);
  G8Args g{A, lda, B, ldb, M, N, K, kps};
  hipLaunchKernelGGL(gemm256_kernel, dim3(tiles, 1, z), dim3(G8_THREADS), 0, s, g, ep);
}

}  // namespace tam
