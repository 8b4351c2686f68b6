// tiresias_amd — grouped weight-gradient GEMM: many independent
//   C_p[M_p][N_p] += A_p^T B_p        (A_p = dY_p [K_p][M_p], B_p = X_p [K_p][N_p])
// problems of one backward pass in ONE launch, plus the bias gradients
// (colsum_p[m] += sum_k A_p[k][m]) of the same dY operands.
//
// Why (Transformer-base, d = 512): every Linear layer's dW = dY^T X is a
// 512..2048 x 512 x 4096 GEMM of 16-64 128^2 tiles. Issued one per layer each
// underfills the 256 CUs (the per-shape route table picked 64x64 igemm tiles
// for them: 60 launches, ~33 us each, ~50 % of the step's GPU time). All of a
// step's weight gradients are independent of each other, so the trainer
// defers them (functional.py DeferredWgrad) and issues them here as one grid
// of ~2700 128^2 tiles of the LDS-DMA gemm8p core (gemm8p.h), which fills the
// chip for ~5 waves.
//
// Grid layout: blocks [0, ncs) are column-sum blocks (64 bias columns of one
// problem each, 256 threads = 8 x 16-B column chunks x 32 row lanes, a plain
// += by the single owner -- deterministic, no atomics); blocks [ncs, ...)
// are GEMM tiles, problem p owning tiles [t0_p, t0_{p+1}). The memory-bound
// column sums are dispatched first, beside the first MFMA wave.
#include <cstdlib>

#include "tam/launch.h"
#include "tam/tiles.h"
#include "tam/gemm8p.h"

namespace tam {

constexpr int P8G_MAX = 64;   // problems per launch (kernel-argument budget: 64 x 64 B)

struct P8GProb {
  const bf16_t* A;   // [K][M] M-major (dY), contiguous
  const bf16_t* B;   // [K][N] N-major (X), contiguous
  float* C;          // [M][N] fp32, stored (mode 0) or accumulated (mode 1)
  float* bias;       // optional: [M] += column sums of A
  int M, N, K;
  int t0;            // first GEMM tile (relative to the GEMM part of the grid)
  int c0;            // first column-sum block
  int mode;          // 0: C = A^T B (a weight's first gradient write of the step), 1: C +=
  int ntiles;        // output tiles
  int kps;           // K-tiles per slice; slices = (tiles owned) / ntiles
};

struct P8Group {
  P8GProb p[P8G_MAX];
  int n;
  int ncs;           // column-sum blocks in all
};

// 64 columns [m0, m0 + 64) of A summed over all K rows by one block
// (8 x 16-B column chunks x blockDim/8 row lanes, 4 loads in flight each)
__device__ __forceinline__ void gg_colsum(const P8GProb& pr, int blk, float* red) {
  const int m0 = blk * 64;
  const int tid = threadIdx.x, cg = tid & 7, rl = tid >> 3;
  const int RL = blockDim.x >> 3;
  const int col = m0 + cg * 8;
  float s[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = 0.f;
  if (col < pr.M) {
    const bf16_t* p = pr.A + col;
    int r = rl;
    for (; r + 3 * RL < pr.K; r += 4 * RL) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *(const uint4*)(p + (long)(r + RL * u) * pr.M);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s[2 * e] += bf2f((bf16_t)(w[e] & 0xffff));
          s[2 * e + 1] += bf2f((bf16_t)(w[e] >> 16));
        }
      }
    }
    for (; r < pr.K; r += RL) {
      const uint4 v = *(const uint4*)(p + (long)r * pr.M);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s[2 * e] += bf2f((bf16_t)(w[e] & 0xffff));
        s[2 * e + 1] += bf2f((bf16_t)(w[e] >> 16));
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl * 64 + cg * 8 + e] = s[e];   // [row lane][64 columns]
  __syncthreads();
  if (tid < 64 && m0 + tid < pr.M) {
    float t = 0.f;
    for (int k = 0; k < RL; ++k) t += red[k * 64 + tid];
    pr.bias[m0 + tid] += t;
  }
}

template <int BM, int BN, int WNW>
__global__ void __launch_bounds__(64 * 2 * WNW, (BM == 256 ? 1 : 2)) gemm8p_grouped_kernel(P8Group g) {
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  if (bid < g.ncs) {
    __shared__ float cs_red[64 * 64];
    int c = 0;
    while (c + 1 < g.n && bid >= g.p[c + 1].c0) ++c;
    gg_colsum(g.p[c], bid - g.p[c].c0, cs_red);
    return;
  }
  const int t = bid - g.ncs;
  int c = 0;
  while (c + 1 < g.n && t >= g.p[c + 1].t0) ++c;
  const P8GProb& pr = g.p[c];
  // a long-K problem is split over K: slice-major unit order, so the
  // consecutive blocks of one XCD (xcd_remap) are tiles of ONE K-slice and
  // share its A / B panels in L2; the slices meet in fp32 atomics (mode 2)
  const int u = t - pr.t0;
  const int tile = u % pr.ntiles, kz = u / pr.ntiles;
  const bool split = pr.kps < pr.K / P8_BK;
  P8Args a{pr.A, (long)pr.M, pr.B, (long)pr.N, pr.M, pr.N, pr.K, pr.kps, 4};
  Epi ep;
  ep.c = pr.C;
  ep.ldc = pr.N;
  ep.c_f32 = 1;
  ep.mode = split ? 2 : pr.mode;
  gemm8p_body<BM, BN, WNW, false, false>(a, ep, tile, kz);
}

// tile of the grouped launch: 128 (128^2, 4 waves, 2 blocks / CU; default)
// or 256 (256^2, 8 waves, 1 block / CU); TAM_GROUPED_TILE overrides. The
// Transformer step measured 5.46 ms with 128 vs 5.79 ms with 256
// (profiles/r4/grouped_wgrad.md)
static int g_gg_tile = [] {
  const char* e = getenv("TAM_GROUPED_TILE");
  return e ? atoi(e) : 128;
}();
TAM_KNOB(g_gg_tile)
void gemm_grouped_tile(int t) { g_gg_tile = t == 256 ? 256 : 128; }

// K-split of long-K problems: a problem of more than 2x this many K-tiles
// (64 deep each) is cut into slices of about this many (<= 32 slices) whose
// partial tiles meet in fp32 atomics -- accumulate-mode (1) problems only.
// ResNet-50's 1x1-conv weight gradients are 128..2048 x 128..2048 GEMMs
// over K = 3136..200704 output pixels: unsplit, a 4-tile problem would run
// ~800 K-tiles on 4 CUs. 0: never split. The Transformer / GNMT problems
// (K = 3136..4096) stay whole.
static int g_gg_split_kt = [] {
  const char* e = getenv("TAM_GROUPED_SPLIT_KT");
  return e ? atoi(e) : 64;
}();
TAM_KNOB(g_gg_split_kt)

static int gg_kps(int K, int mode) {
  const int kt = K / P8_BK;
  if (g_gg_split_kt <= 0 || mode != 1 || kt <= 2 * g_gg_split_kt) return kt;
  int sk = cdiv(kt, g_gg_split_kt);
  if (sk > 32) sk = 32;
  return cdiv(kt, sk);
}

// problems: A [K][lda] (M-major), B [K][ldb] (N-major), C [M][N] fp32 = or +=,
// bias [M] += colsum(A) or null. Host checks the gemm8p conditions (K % 64,
// M, N >= 128 and % 8, lda / ldb % 8) -- the caller routes anything else to
// the per-problem gemm(). Launches ceil(n / P8G_MAX) grids.
void gemm_wgrad_grouped(const GGProblem* probs, int n, hipStream_t s) {
  const int T = g_gg_tile == 128 ? 128 : 256;
  for (int base = 0; base < n; base += P8G_MAX) {
    P8Group g{};
    const int m = n - base < P8G_MAX ? n - base : P8G_MAX;
    int tiles = 0, cs = 0;
    for (int i = 0; i < m; ++i) {
      const GGProblem& q = probs[base + i];
      P8GProb& p = g.p[i];
      p.A = q.A; p.B = q.B; p.C = q.C; p.bias = q.bias;
      p.M = q.M; p.N = q.N; p.K = q.K;
      p.mode = q.mode;
      p.t0 = tiles;
      p.c0 = cs;
      p.ntiles = cdiv(q.M, T) * cdiv(q.N, T);
      p.kps = gg_kps(q.K, q.mode);
      tiles += p.ntiles * cdiv(q.K / P8_BK, p.kps);
      if (q.bias) cs += cdiv(q.M, 64);
    }
    // (a bias-less problem owns no column-sum blocks: its c0 equals the next
    // problem's, and the device scan picks the LAST problem with c0 <= bid)
    g.n = m;
    g.ncs = cs;
    if (tiles + cs == 0) continue;
    if (T == 128)
      hipLaunchKernelGGL((gemm8p_grouped_kernel<128, 128, 2>), dim3((unsigned)(tiles + cs)), dim3(256), 0, s, g);
    else
      hipLaunchKernelGGL((gemm8p_grouped_kernel<256, 256, 4>), dim3((unsigned)(tiles + cs)), dim3(512), 0, s, g);
  }
}

bool gemm_wgrad_grouped_ok(int M, int N, int K, long lda, long ldb) {
  // contiguous operands only (lda == M, ldb == N: the problem table packs no strides)
  return lda == M && ldb == N && gemm8p_ok(false, false, M, N, K, lda, ldb) &&
         (long)K * (M > N ? M : N) < (1L << 31);
}

}  // namespace tam
