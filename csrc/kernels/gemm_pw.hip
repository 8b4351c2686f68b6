// tiresias_amd — short-K / narrow-N GEMM for pointwise (1x1, stride-1)
// convolutions over many pixels: C[M][N] = A[M][K] . B[N][K]^T, bf16 in and
// out, K <= 256, N <= 256, K * N <= 16384. ResNet-50's 56x56 bottleneck convs
// at batch 64 (M = 200704 pixels, K / N in {64, 128, 256}) are memory-bound:
// the 64x64 igemm tiles re-read every A row once per 64 output columns and
// leave the block's loads, MFMAs and stores in one dependent chain, so they ran
// at ~3 TB/s (profiles/r6/pw_conv.md).
//
// MI355X-first structure:
//  * The whole B (the 1x1 weight, <= 32 KiB) is staged into LDS ONCE per
//    block (padded rows: the 16-lane fragment reads hit 16 banks); blocks are
//    persistent over 64-row M-tiles, so each A row is read exactly once.
//  * Wave w owns rows 16w..16w+15 of a tile and ALL N columns (N/16 MFMA
//    tiles of v_mfma_f32_16x16x32_bf16); its A fragments come straight from
//    global memory (16 B per lane per k-step: row = lane % 16, k = 8 (lane/16))
//    and the NEXT tile's fragments are loaded before this tile's MFMAs.
//  * Epilogue through a per-wave padded LDS slab: 16-B row chunks out, the
//    ReLU-backward mask (dgrad) read in the same 16-B units, and the
//    BatchNorm statistics of the stored values (sum | sum of squares per
//    channel) accumulated in registers across all of the block's tiles, then
//    one fp64 atomic per channel per block into shard blockIdx % BN_SHARDS
//    (the layout of every conv epilogue, Epi::stats).
#include "tam/launch.h"
#include "tam/kernels.h"

namespace tam {

struct PwArgs {
  const bf16_t* A;
  long lda;
  const bf16_t* B;
  long ldb;
  bf16_t* C;
  long ldc;
  long M;
  const bf16_t* mask;   // zero where mask <= 0 (relu backward), or null
  long ldm;
  double* stats;        // fp64 [BN_SHARDS][2N], or null
  int relu;
};

template <int K, int N>
__global__ void __launch_bounds__(256, 2) gemm_pw_kernel(PwArgs a) {
  constexpr int KT = K / 32, NT = N / 16;
  constexpr int BLD = K + 8;                    // padded B row (bf16): 16-B shift per row
  constexpr int SLD = N + 8;                    // padded slab row
  constexpr int CPR = N / 8;                    // 16-B chunks per output row
  constexpr int RPU = 64 / CPR;                 // rows covered per 64-lane store instruction
  constexpr int S = 16 / RPU;                   // 16-B store chunks per lane per tile
  static_assert(K % 32 == 0 && N % 16 == 0 && CPR <= 64 && 64 % CPR == 0, "gemm_pw shape");
  __shared__ __attribute__((aligned(16))) bf16_t Bs[N * BLD];
  __shared__ __attribute__((aligned(16))) bf16_t slab[4][16 * SLD];
  __shared__ float red[4][2 * N];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;

  // B -> LDS once (16-B chunks)
  for (int i = tid; i < N * (K / 8); i += 256) {
    const int n = i / (K / 8), c = (i % (K / 8)) * 8;
    *(uint4*)(Bs + n * BLD + c) = *(const uint4*)(a.B + (long)n * a.ldb + c);
  }
  __syncthreads();

  const long ntiles = (a.M + 63) / 64;
  const int r16 = lane & 15, koff = 8 * (lane >> 4);
  // rows past M read row M-1 (never stored): unpredicated loads keep the
  // group's code straight-line for the compiler's counted waits
  auto load_a = [&](long mt, s16x8_t (&f)[KT]) {
    long m = mt * 64 + 16 * w + r16;
    m = m < a.M ? m : a.M - 1;
#pragma unroll
    for (int ks = 0; ks < KT; ++ks) f[ks] = *(const s16x8_t*)(a.A + m * a.lda + 32 * ks + koff);
  };
  float ssum[8], ssq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) ssum[e] = ssq[e] = 0.f;
  const bool stats = a.stats != nullptr;
  const int ch = lane % CPR;                    // this lane's 8-channel chunk in the store pass

  // Software pipeline over the block's tiles: the NEXT tile's A fragments
  // (and, for narrow outputs, its mask chunks) are issued before this tile's
  // MFMAs and stores. Loads are unpredicated (rows past M read row M-1) and
  // stores too (rows past M recompute row M-1 from the same clamped A row and
  // store the identical values there), so every lane issues the same vector-
  // memory instructions in every tile: the compiler's in-order counted waits
  // then retire exactly the current tile's loads while the next tile's stay
  // in flight. Two register sets, alternating (no loop-carried copies).
  constexpr bool MPRE = S <= 2;
  struct Regs {
    s16x8_t af[KT];
    uint4 mk[MPRE ? S : 1];
  };
  auto issue = [&](long mt, Regs& r) {
    load_a(mt, r.af);
    if constexpr (MPRE) {
      if (a.mask) {
#pragma unroll
        for (int u = 0; u < S; ++u) {
          long m = mt * 64 + 16 * w + u * RPU + lane / CPR;
          m = m < a.M ? m : a.M - 1;
          r.mk[u] = *(const uint4*)(a.mask + m * a.ldm + ch * 8);
        }
      }
    }
  };
  auto tile = [&](long mt, Regs& cur, Regs& nxt) {
    const long mn = mt + gridDim.x < ntiles ? mt + gridDim.x : mt;   // (re-reads the last tile)
    issue(mn, nxt);
    __builtin_amdgcn_sched_barrier(0);
    f32x4_t acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KT; ++ks)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const s16x8_t bf = *(const s16x8_t*)(Bs + (16 * j + r16) * BLD + 32 * ks + koff);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, cur.af[ks]),
                                                         __builtin_bit_cast(bf16x8_t, bf), acc[j], 0, 0, 0);
      }
    // C/D map: col = lane & 15, row = 4 (lane >> 4) + r
    bf16_t* sl = slab[w];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[j][r];
        if (a.relu) v = fmaxf(v, 0.f);
        sl[(4 * (lane >> 4) + r) * SLD + 16 * j + r16] = f2bf(v);
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < S; ++u) {
      const int lr = u * RPU + lane / CPR;
      const long m = mt * 64 + 16 * w + lr;
      const long ms = m < a.M ? m : a.M - 1;
      uint4 v = *(const uint4*)(sl + lr * SLD + ch * 8);
      if (a.mask) {
        uint4 mk;
        if constexpr (MPRE) mk = cur.mk[u];
        else mk = *(const uint4*)(a.mask + ms * a.ldm + ch * 8);
        const uint32_t* mw = (const uint32_t*)&mk;
        uint32_t* vw = (uint32_t*)&v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t m2 = mw[e];
          const bool lo = (m2 & 0x8000u) == 0 && (m2 & 0x7fffu) != 0;
          const bool hi = (m2 & 0x80000000u) == 0 && (m2 & 0x7fff0000u) != 0;
          vw[e] &= (lo ? 0x0000ffffu : 0u) | (hi ? 0xffff0000u : 0u);
        }
      }
      *(uint4*)(a.C + ms * a.ldc + ch * 8) = v;
      if (stats) {
        const float inr = m < a.M ? 1.f : 0.f;   // a clamped duplicate row adds nothing
        const uint32_t* vw = (const uint32_t*)&v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = __uint_as_float(vw[e] << 16) * inr, hi = __uint_as_float(vw[e] & 0xffff0000u) * inr;
          ssum[2 * e] += lo; ssq[2 * e] += lo * lo;
          ssum[2 * e + 1] += hi; ssq[2 * e + 1] += hi * hi;
        }
      }
    }
  };
  Regs r0, r1;
  long mt = blockIdx.x;
  if (mt < ntiles) issue(mt, r0);
  for (; mt < ntiles; mt += 2 * (long)gridDim.x) {
    tile(mt, r0, r1);
    if (mt + gridDim.x < ntiles) tile(mt + gridDim.x, r1, r0);
  }
  if (!stats) return;
  // lanes sharing a chunk (lane % CPR) -> one value per chunk per wave, then
  // the 4 waves in LDS, one fp64 atomic per channel per block
#pragma unroll
  for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      ssum[e] += __shfl_xor(ssum[e], o, 64);
      ssq[e] += __shfl_xor(ssq[e], o, 64);
    }
  if (lane < CPR) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[w][lane * 8 + e] = ssum[e];
      red[w][N + lane * 8 + e] = ssq[e];
    }
  }
  __syncthreads();
  double* sh = a.stats + (long)(blockIdx.x % BN_SHARDS) * 2 * N;
  for (int e = tid; e < 2 * N; e += 256)
    unsafeAtomicAdd(sh + e, (double)(red[0][e] + red[1][e] + red[2][e] + red[3][e]));
}

// 1 (default): pointwise convs of eligible shapes take this kernel; 0: the
// dense GEMM route (A/B). TAM_CONV_PW
static int g_conv_pw = [] {
  const char* e = getenv("TAM_CONV_PW");
  return e ? atoi(e) : 1;
}();
TAM_KNOB(g_conv_pw)
void gemm_pw_policy(int on) { g_conv_pw = on; }

bool gemm_pw_ok(long M, int N, int K, long lda, long ldb, long ldc) {
  if (!g_conv_pw || M < 65536) return false;   // memory-bound regime only (many pixels)
  // K * N <= 16384: the whole weight in LDS with two blocks per CU (the
  // 128 x 256 / 256 x 128 instantiations fit only one and measured 2x slower
  // than the dense route, profiles/r6/pw_conv.md)
  const bool kn = (K == 64 || K == 128 || K == 256) && (N == 64 || N == 128 || N == 256) && K * N <= 16384;
  return kn && lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0;
}

// persistent grid: the resident blocks of the whole device (occupancy of this
// instantiation x CUs, queried once), or fewer when there are fewer tiles
template <int K, int N>
static void pw_launch(const PwArgs& a, hipStream_t s) {
  static const long resident = [] {
    int dev = 0, per_cu = 1;
    hipDeviceProp_t prop;
    TAM_HIP_CHECK(hipGetDevice(&dev));
    TAM_HIP_CHECK(hipGetDeviceProperties(&prop, dev));
    TAM_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gemm_pw_kernel<K, N>, 256, 0));
    return (long)(per_cu < 1 ? 1 : per_cu) * prop.multiProcessorCount;
  }();
  const long ntiles = (a.M + 63) / 64;
  const long blocks = ntiles < resident ? ntiles : resident;
  hipLaunchKernelGGL((gemm_pw_kernel<K, N>), dim3((unsigned)blocks), dim3(256), 0, s, a);
}

// C[M][N] (bf16, ldc) = A[M][K] (lda) . B[N][K]^T (ldb); mask / stats / relu
// as in Epi. Returns false (nothing launched) when the shape is not eligible.
bool gemm_pw(const bf16_t* A, long lda, const bf16_t* B, long ldb, bf16_t* C, long ldc, long M, int N, int K,
             const bf16_t* mask, long ldm, double* stats, int relu, hipStream_t s) {
  if (!gemm_pw_ok(M, N, K, lda, ldb, ldc)) return false;
  if (mask && ldm % 8 != 0) return false;
  const PwArgs a{A, lda, B, ldb, C, ldc, M, mask, ldm, stats, relu};
  switch (K * 1000 + N) {
    case 64064: pw_launch<64, 64>(a, s); return true;
    case 64128: pw_launch<64, 128>(a, s); return true;
    case 64256: pw_launch<64, 256>(a, s); return true;
    case 128064: pw_launch<128, 64>(a, s); return true;
    case 128128: pw_launch<128, 128>(a, s); return true;
    case 256064: pw_launch<256, 64>(a, s); return true;
    default: return false;
  }
}

}  // namespace tam
