// tiresias_amd — generic MFMA implicit-GEMM core for gfx950.
//
//   C[M,N] (+)= alpha * sum_k A(m,k) * B(k,n)        bf16 in, fp32 accumulate
//
// One template serves plain GEMM (all four operand majorities) and the three
// NHWC convolution passes (fwd / dgrad / wgrad): only the operand *loaders*
// differ. Design (CDNA4-first, see cdna_hip_programming.md §5):
//   * 256 threads = 4 waves in a 2x2 grid; each wave owns a (BM/2)x(BN/2)
//     sub-tile built from v_mfma_f32_16x16x32_bf16 (16x16 outputs, K=32).
//   * BK = 64; A and B tiles are register-staged (16-byte global loads issued
//     *before* the MFMA phase of the current tile, written to the other LDS
//     buffer *after* it: async-STAGE split, guide T14) into a 2-deep LDS ring,
//     one barrier per K-tile.
//   * K-major operands live in LDS as [rows][64] bf16 with the 16-B chunk
//     XOR-swizzled by (row>>1)&7 -> ds_read_b128 fragment reads conflict-free
//     for the gfx950 ds_read_b128 lane groups (checked exhaustively offline).
//   * MN-major operands (the transposed operand of dgrad/wgrad GEMMs) live in
//     LDS as [64][cols] and are read with ds_read_b64_tr_b16 (hardware
//     transpose, guide T10), 8-B chunk XOR-swizzled per row so both the 16-B
//     register-staged writes and the transposed reads are conflict-free.
//   * Workgroup ids are XCD-remapped (bijective, T1) and then grouped along M
//     so consecutive tiles on one XCD share A panels in that XCD's L2.
//   * Split-K over blockIdx.z with fp32 atomics for reduction-heavy shapes
//     (conv wgrad, Linear dW).
#pragma once
#include "tam/common.h"

namespace tam {

constexpr int IG_BK = 64;
constexpr int IG_THREADS = 256;

struct Epi {
  void* c = nullptr;        // output base
  long ldc = 0;             // output row stride (elements)
  int c_f32 = 0;            // 1: fp32 output, 0: bf16 output
  int mode = 0;             // 0: store, 1: accumulate (C += .), 2: fp32 atomic add
  const bf16_t* bias = nullptr;  // per-column bias (bf16), added once
  int relu = 0;             // apply max(.,0) after bias
  const bf16_t* mask = nullptr;  // relu-backward mask: zero where mask<=0
  long ldm = 0;
  float alpha = 1.f;
  long zstride = 0;
  // conv_dma bf16 epilogue only: per-channel BatchNorm sums of the stored
  // outputs, fp64 [BN_SHARDS][2N] (sum | sum of squares), accumulated with
  // device-scope atomics into shard (M-tile % BN_SHARDS); the caller zeroes them
  double* stats = nullptr;
  // conv_dma bf16 epilogue only, with stats: the stored tile is the gradient
  // d of a BatchNorm OUTPUT whose input was bnx (same [rows][N] layout):
  // the sums become sum(d) | sum(d * (bnx - mean) * rstd) -- the
  // BN-backward reduction, read from the dgrad epilogue instead of a pass
  const bf16_t* bnx = nullptr;
  const float* bnmean = nullptr;
  const float* bnrstd = nullptr;
  // igemm with an M-major A only: colsum_a[m] += sum_k A[k][m] (fp32 no-return
  // atomics, one per column per K-split) -- a Linear layer's bias gradient
  // from the weight-gradient GEMM's own A loads (dW = dY^T X, db = colsum(dY))
  float* colsum_a = nullptr;
};

// ---------------------------------------------------------------------------
// LDS image addressing
// ---------------------------------------------------------------------------
// K-major tile image: [rows][64] bf16, 128-B rows, 16-B chunk c of row r at
// chunk (c ^ ((r>>1)&7)).
__device__ __forceinline__ int kmaj_off(int r, int c16) {
  return r * 128 + ((c16 ^ ((r >> 1) & 7)) << 4);
}
// MN-major tile image: [64][COLS] bf16. 8-B chunk index XOR-ed with a per-row
// value (multiple of 4 so 16-B pairs stay contiguous).
template <int COLS>
__device__ __forceinline__ int mnmaj_swz(int r) {
  if constexpr (COLS == 128) return 4 * ((r & 3) | (((r >> 3) & 1) << 2));
  else return (4 * ((r >> 1) & 1)) ^ (8 * ((r >> 3) & 1));   // COLS == 64
}
template <int COLS>
__device__ __forceinline__ int mnmaj_off(int r, int c8) {
  return r * (COLS * 2) + ((c8 ^ mnmaj_swz<COLS>(r)) << 3);
}

typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;

template <int COLS>
__device__ __forceinline__ s16x8_t read_frag_mn(const char* tile, int lane, int kbase, int colbase) {
  // lane (g = lane>>4, t = lane&15, q = t>>2, p = t&3) supplies row
  // kbase + 8g + 4h + q, columns colbase + 4p..4p+3; receives column
  // colbase + t, k = kbase + 8g + 4h + q  (q = element index)
  const int g = lane >> 4, t = lane & 15, q = t >> 2, p = t & 3;
  const int c8 = (colbase >> 2) + p;
  const int r0 = kbase + 8 * g + q;
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(tile + mnmaj_off<COLS>(r0, c8)));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(tile + mnmaj_off<COLS>(r0 + 4, c8)));
  s16x8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

__device__ __forceinline__ s16x8_t read_frag_k(const char* tile, int lane, int rowbase, int kk) {
  const int r = rowbase + (lane & 15);
  const int c = 4 * kk + (lane >> 4);
  return *(const s16x8_t*)(tile + kmaj_off(r, c));
}

__device__ __forceinline__ uint4 ld16(const bf16_t* p) { return *(const uint4*)p; }

// ---------------------------------------------------------------------------
// Loaders. Each exposes:
//   static constexpr bool kKMajor;
//   init(int tile0, int tid)  -- per-thread precompute for this block's tile
//   uint4 load(int pass, int kglob)
// K-major, ROWS-row tile: thread t, pass p -> row (t>>3)+32p, k = kglob
//   (kglob = k0 + 8*(t&7) is computed by the kernel).
// MN-major, COLS-col tile: thread t, pass p -> k-row kglob (= k0 + t/CPR +
//   p*256/CPR computed by the kernel), column chunk (t%CPR)*8.
// ---------------------------------------------------------------------------

// 16 zero bytes: the source of out-of-range loads (zero-initialised)
static __device__ __attribute__((aligned(16))) uint4 g_ig_zero[1];

// Dense K-major: elem(row, k) = p[row*ld + k]
template <int ROWS>
struct LdKMajor {
  static constexpr bool kKMajor = true;
  static constexpr int P = ROWS / 32;
  const bf16_t* p; long ld; int rows; int K;
  const bf16_t* rp[P]; bool rv[P];
  __device__ void init(int row0, int tid) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      int r = row0 + (tid >> 3) + 32 * i;
      rv[i] = r < rows;
      rp[i] = p + (long)(rv[i] ? r : 0) * ld;
    }
  }
  // unpredicated: an out-of-range element reads 16 zero bytes of g_ig_zero
  // (an address select BEFORE the load, no select on its data), so the load
  // issues with no exec-mask branch around it and nothing waits on it early
  __device__ uint4 load(int i, int k) const {
    const bool ok = rv[i] && k < K;
    return ld16(ok ? rp[i] + k : (const bf16_t*)g_ig_zero);
  }
};

// Dense MN-major: elem(k, col) = p[k*ld + col]
template <int COLS>
struct LdMNMajor {
  static constexpr bool kKMajor = false;
  const bf16_t* p; long ld; int cols; int K;
  int col; bool cv;
  __device__ void init(int col0, int tid) {
    col = col0 + (tid % (COLS / 8)) * 8;
    cv = col < cols;
  }
  __device__ uint4 load(int, int k) const {     // unpredicated, as LdKMajor
    const bool ok = cv && k < K;
    return ld16(ok ? p + (long)k * ld + col : (const bf16_t*)g_ig_zero);
  }
};

struct ConvGeom {
  int N, H, W, C;      // input NHWC
  int K, R, S;         // filters [K][R][S][C]
  int P, Q;            // output spatial
  int stride, pad, dil;
};

// floor(n / d) for 0 <= n < 2^31 by a multiply-high (Granlund-Montgomery,
// N = 31: mul = ceil(2^(31 + l) / d) < 2^32, l = ceil(log2 d)), built on the
// host once per launch. The im2col loaders below decode a pixel or a (tap,
// channel) index for EVERY 16-B load; with runtime '/' and '%' that was ~20
// VALU per division, four to six divisions per load (PMC: 22-24 VALU per
// MFMA in the gather igemm, VALU utilisation 0.5-1.0)
struct FastDiv {
  uint32_t d = 1, mul = 0;
  int sh = 0;
  FastDiv() = default;
  explicit FastDiv(int dv) : d(dv < 1 ? 1u : (uint32_t)dv) {
    if (d == 1) return;
    int l = 0;
    while ((1u << l) < d) ++l;                     // d >= 2: l >= 1
    mul = (uint32_t)(((1ull << (31 + l)) + d - 1) / d);
    sh = l - 1;
  }
  __device__ __forceinline__ int div(int n) const {
    return d == 1 ? n : (int)(__umulhi((uint32_t)n, mul) >> sh);
  }
};

// conv fwd A operand: rows = output pixels (n,p,q), k = (r,s,c) c fastest.
// K-major gather from X (requires C % 8 == 0).
template <int ROWS>
struct LdConvFwdA {
  static constexpr bool kKMajor = true;
  static constexpr int P_ = ROWS / 32;
  const bf16_t* x; ConvGeom g; int M; int Kdim;
  FastDiv fc, fs;      // by C, by S (host: with_divs)
  int nb[P_], h0[P_], w0[P_];
  LdConvFwdA& with_divs() { fc = FastDiv(g.C); fs = FastDiv(g.S); return *this; }
  __device__ void init(int row0, int tid) {
#pragma unroll
    for (int i = 0; i < P_; ++i) {
      int m = row0 + (tid >> 3) + 32 * i;
      if (m < M) {
        int q = m % g.Q; int t = m / g.Q; int pp = t % g.P; int n = t / g.P;
        nb[i] = n; h0[i] = pp * g.stride - g.pad; w0[i] = q * g.stride - g.pad;
      } else {
        nb[i] = -1; h0[i] = 0; w0[i] = 0;
      }
    }
  }
  __device__ uint4 load(int i, int k) const {   // unpredicated (zero page), as LdKMajor
    const int rs = fc.div(k), c = k - rs * g.C, r = fs.div(rs), s = rs - r * g.S;
    const int h = h0[i] + r * g.dil, w = w0[i] + s * g.dil;
    const bool ok = nb[i] >= 0 && k < Kdim && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
    return ld16(ok ? x + (((long)nb[i] * g.H + h) * g.W + w) * g.C + c : (const bf16_t*)g_ig_zero);
  }
};

// conv dgrad A operand: rows = input pixels (n,h,w), k = (r,s,ko) ko fastest.
// dX(n,h,w,c) = sum dY(n,p,q,ko) W(ko,r,s,c) over (h+pad-r*dil) = p*stride.
// K-major gather from dY (requires K % 8 == 0).
template <int ROWS>
struct LdConvDgradA {
  static constexpr bool kKMajor = true;
  static constexpr int P_ = ROWS / 32;
  const bf16_t* dy; ConvGeom g; int M; int Kdim;
  FastDiv fk, fs, fst;   // by K, by S, by stride (host: with_divs)
  int nb[P_], hh[P_], ww[P_];
  LdConvDgradA& with_divs() { fk = FastDiv(g.K); fs = FastDiv(g.S); fst = FastDiv(g.stride); return *this; }
  __device__ void init(int row0, int tid) {
#pragma unroll
    for (int i = 0; i < P_; ++i) {
      int m = row0 + (tid >> 3) + 32 * i;
      if (m < M) {
        int w = m % g.W; int t = m / g.W; int h = t % g.H; int n = t / g.H;
        nb[i] = n; hh[i] = h + g.pad; ww[i] = w + g.pad;
      } else {
        nb[i] = -1; hh[i] = 0; ww[i] = 0;
      }
    }
  }
  __device__ uint4 load(int i, int k) const {   // unpredicated (zero page), as LdKMajor
    const int rs = fk.div(k), ko = k - rs * g.K, r = fs.div(rs), s = rs - r * g.S;
    const int pn = hh[i] - r * g.dil, qn = ww[i] - s * g.dil;
    const int pp = fst.div(pn < 0 ? 0 : pn), qq = fst.div(qn < 0 ? 0 : qn);
    const bool ok = nb[i] >= 0 && k < Kdim && pn >= 0 && qn >= 0 && pp * g.stride == pn &&
                    qq * g.stride == qn && pp < g.P && qq < g.Q;
    return ld16(ok ? dy + (((long)nb[i] * g.P + pp) * g.Q + qq) * g.K + ko : (const bf16_t*)g_ig_zero);
  }
};

// conv wgrad B operand: k-rows = output pixels m=(n,p,q) (reduction), cols =
// (r,s,c) c fastest. MN-major gather from X (requires C % 8 == 0).
template <int COLS>
struct LdConvWgradB {
  static constexpr bool kKMajor = false;
  const bf16_t* x; ConvGeom g; int Mred; int Ncols;
  FastDiv fq, fp;      // by Q, by P (host: with_divs)
  int cr, cs, cc; bool cv;
  LdConvWgradB& with_divs() { fq = FastDiv(g.Q); fp = FastDiv(g.P); return *this; }
  __device__ void init(int col0, int tid) {
    int col = col0 + (tid % (COLS / 8)) * 8;
    cv = col < Ncols;
    int c = col % g.C; int rs = col / g.C;
    cc = c; cs = rs % g.S; cr = rs / g.S;
  }
  __device__ uint4 load(int, int m) const {    // unpredicated (zero page), as LdKMajor
    const int t = fq.div(m), q = m - t * g.Q, n = fp.div(t), pp = t - n * g.P;
    const int h = pp * g.stride - g.pad + cr * g.dil, w = q * g.stride - g.pad + cs * g.dil;
    const bool ok = cv && m < Mred && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
    return ld16(ok ? x + (((long)n * g.H + h) * g.W + w) * g.C + cc : (const bf16_t*)g_ig_zero);
  }
};

// ---------------------------------------------------------------------------
// The kernel
// ---------------------------------------------------------------------------
template <class L, int EXT>
struct Stager {
  // EXT = tile extent along the operand's M (or N) dimension
  static constexpr int P = EXT / 32;   // 16-B loads per thread per K-tile
  __device__ static void fetch(const L& l, uint4 (&r)[P], int k0, int tid) {
    if constexpr (L::kKMajor) {
      const int k = k0 + 8 * (tid & 7);
#pragma unroll
      for (int i = 0; i < P; ++i) r[i] = l.load(i, k);
    } else {
      constexpr int CPR = EXT / 8, RPP = IG_THREADS / CPR;
#pragma unroll
      for (int i = 0; i < P; ++i) r[i] = l.load(i, k0 + tid / CPR + i * RPP);
    }
  }
  __device__ static void store(char* tile, const uint4 (&r)[P], int tid) {
    if constexpr (L::kKMajor) {
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const int row = (tid >> 3) + 32 * i, c = tid & 7;
        *(uint4*)(tile + kmaj_off(row, c)) = r[i];
      }
    } else {
      constexpr int CPR = EXT / 8, RPP = IG_THREADS / CPR;
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const int row = tid / CPR + i * RPP, c16 = tid % CPR;
        *(uint4*)(tile + mnmaj_off<EXT>(row, 2 * c16)) = r[i];
      }
    }
  }
  __device__ static s16x8_t frag(const char* tile, int lane, int base, int kk) {
    if constexpr (L::kKMajor) return read_frag_k(tile, lane, base, kk);
    else return read_frag_mn<EXT>(tile, lane, 32 * kk, base);
  }
};

// NPF: register-staged K-tiles in flight. 1: the next tile's loads have ONE
// K-tile of MFMA work to land (the conv loaders, whose address math is
// heavier); NPF > 1: tiles t+1 .. t+NPF are in flight while tile t computes
// (NPF register sets, the loop unrolled by NPF so every set index is a
// compile-time constant) -- the plain small-tile GEMMs with deep K (weight
// gradients: 64 K-tiles of 8 MFMAs per wave) are load-latency bound at NPF 1.
template <int BM, int BN, class LA, class LB, int NPF = 1>
__global__ void __launch_bounds__(IG_THREADS, 2)
igemm_kernel(LA la, LB lb, int M, int N, int K, int ktiles_per_split, Epi ep) {
  constexpr int BK = IG_BK;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int TM = BM / 32, TN = BN / 32;   // 16x16 MFMA tiles per wave
  __shared__ __attribute__((aligned(16))) char smem[2 * (A_BYTES + B_BYTES)];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int grp = bid / per_group;
  const int first_m = grp * GROUP;
  const int gsize = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (bid % per_group) % gsize;
  const int tn = (bid % per_group) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  const int ktiles = (K + BK - 1) / BK;
  const int kt0 = blockIdx.z * ktiles_per_split;
  const int kt1 = min(ktiles, kt0 + ktiles_per_split);

  la.init(m0, tid);
  lb.init(n0, tid);

  using SA = Stager<LA, BM>;
  using SB = Stager<LB, BN>;
  uint4 ra[NPF][SA::P], rb[NPF][SB::P];
  // fused A column sums (Epi::colsum_a): the column-0 blocks add up the A
  // values they stage (each thread: 8 columns of its own K rows)
  bool csum = false;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (!LA::kKMajor) csum = ep.colsum_a != nullptr && tn == 0;
  auto acc_cols = [&](const uint4 (&rs)[SA::P]) {
    if constexpr (!LA::kKMajor) {
      if (csum) {
#pragma unroll
        for (int i = 0; i < SA::P; ++i) {
          const uint32_t w[4] = {rs[i].x, rs[i].y, rs[i].z, rs[i].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            cs[2 * e] += __uint_as_float(w[e] << 16);
            cs[2 * e + 1] += __uint_as_float(w[e] & 0xffff0000u);
          }
        }
      }
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const char* ta, const char* tb) {
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      s16x8_t fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = SA::frag(ta, lane, wr * (BM / 2) + 16 * i, kk);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = SB::frag(tb, lane, wc * (BN / 2) + 16 * j, kk);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8_t, fa[i]), __builtin_bit_cast(bf16x8_t, fb[j]),
              acc[i][j], 0, 0, 0);
    }
  };
  if (kt0 < kt1) {
    // tile kt0 -> LDS stage 0 (through set 0), then tiles kt0+1 .. kt0+NPF
    // into sets 0 .. NPF-1
    SA::fetch(la, ra[0], kt0 * BK, tid);
    SB::fetch(lb, rb[0], kt0 * BK, tid);
    SA::store(smem, ra[0], tid);
    SB::store(smem + 2 * A_BYTES, rb[0], tid);
    acc_cols(ra[0]);
#pragma unroll
    for (int u = 0; u < NPF; ++u) {
      if (kt0 + 1 + u < kt1) {
        SA::fetch(la, ra[u], (kt0 + 1 + u) * BK, tid);
        SB::fetch(lb, rb[u], (kt0 + 1 + u) * BK, tid);
      }
    }
    __syncthreads();
    for (int kb = kt0; kb < kt1; kb += NPF) {
#pragma unroll
      for (int u = 0; u < NPF; ++u) {
        const int kt = kb + u;            // tile kt + 1 is in set u
        if (kt < kt1) {
          const int cur = (kt - kt0) & 1;
          compute(smem + cur * A_BYTES, smem + 2 * A_BYTES + cur * B_BYTES);
          if (kt + 1 < kt1) {
            SA::store(smem + (cur ^ 1) * A_BYTES, ra[u], tid);
            SB::store(smem + 2 * A_BYTES + (cur ^ 1) * B_BYTES, rb[u], tid);
            acc_cols(ra[u]);
            if (kt + 1 + NPF < kt1) {
              SA::fetch(la, ra[u], (kt + 1 + NPF) * BK, tid);
              SB::fetch(lb, rb[u], (kt + 1 + NPF) * BK, tid);
            }
          }
          __syncthreads();
        }
      }
    }
  }
  if constexpr (!LA::kKMajor) {
    if (csum) {
      // threads t and t' = t + CPR*j hold the same 8 columns: combine in LDS
      // (the stages are free after the loop's last barrier), then one atomic
      // per column
      constexpr int CPR = BM / 8, RPP = IG_THREADS / CPR;
      float* red = (float*)smem;
      if (kt0 >= kt1) __syncthreads();
#pragma unroll
      for (int e = 0; e < 8; ++e) red[tid * 8 + e] = cs[e];
      __syncthreads();
      if (tid < CPR) {
        float t8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) t8[e] = 0.f;
        for (int r = 0; r < RPP; ++r)
#pragma unroll
          for (int e = 0; e < 8; ++e) t8[e] += red[(r * CPR + tid) * 8 + e];
        const int col = m0 + tid * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (col + e < M) atomicAdd(ep.colsum_a + col + e, t8[e]);
      }
      __syncthreads();
    }
  }

  const bool add_bias = ep.bias != nullptr && blockIdx.z == 0;
  // ---- bf16 output: LDS-staged epilogue (whole 16-B row chunks instead of
  // 2-B stores in the MFMA C layout); needs 16-B aligned output rows
  if (!ep.c_f32 && (ep.ldc & 7) == 0 && (((uintptr_t)ep.c) & 15) == 0 &&
      (!ep.mask || ((ep.ldm & 7) == 0 && (((uintptr_t)ep.mask) & 15) == 0))) {
    constexpr int WC = BN / 2, LDW = WC + 8, CPR = WC / 8, NCH = 32 * CPR / 64;
    bf16_t* slab = (bf16_t*)(smem + wid * (32 * LDW * 2));
    if (kt0 >= kt1) __syncthreads();   // (the K loop ends with a barrier otherwise)
    const int cbase = n0 + wc * WC;
    // BatchNorm statistics of the STORED values (Epi::stats; a pointwise
    // conv's output feeding a BN): a lane keeps one 8-column chunk (ch =
    // lane % CPR for every u) over all its rows
    const bool stats = ep.stats != nullptr;
    float ssum[8], ssq[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) ssum[e] = ssq[e] = 0.f;
    float bv[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = cbase + 16 * j + (lane & 15);
      bv[j] = (add_bias && col < N) ? bf2f(ep.bias[col]) : 0.f;
    }
#pragma unroll
    for (int h = 0; h < TM / 2; ++h) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = 2 * h + ii;
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[i][j][r] * ep.alpha + bv[j];
            if (ep.relu) v = fmaxf(v, 0.f);
            slab[(16 * ii + 4 * (lane >> 4) + r) * LDW + 16 * j + (lane & 15)] = f2bf(v);
          }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < NCH; ++u) {
        const int idx = u * 64 + lane, lr = idx / CPR, ch = idx % CPR;
        const int row = m0 + wr * (BM / 2) + 32 * h + lr;
        const int col = cbase + ch * 8;
        if (row >= M || col >= N) continue;
        bf16_t* dst = (bf16_t*)ep.c + (long)row * ep.ldc + col;
        const bf16_t* src = slab + lr * LDW + ch * 8;
        if (col + 8 <= N) {
          uint4 v = *(const uint4*)src;
          uint32_t* vw = (uint32_t*)&v;
          if (ep.mask) {
            const uint4 mk = *(const uint4*)(ep.mask + (long)row * ep.ldm + col);
            const uint32_t* mw = (const uint32_t*)&mk;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const uint32_t m2 = mw[e];
              const bool lo = (m2 & 0x8000u) == 0 && (m2 & 0x7fffu) != 0;
              const bool hi = (m2 & 0x80000000u) == 0 && (m2 & 0x7fff0000u) != 0;
              vw[e] &= (lo ? 0x0000ffffu : 0u) | (hi ? 0xffff0000u : 0u);
            }
          }
          if (ep.mode == 1) {
            const uint4 o = *(const uint4*)dst;
            const uint32_t* ow = (const uint32_t*)&o;
#pragma unroll
            for (int e = 0; e < 4; ++e)
              vw[e] = pack_bf2(bf2f((bf16_t)(vw[e] & 0xffff)) + bf2f((bf16_t)(ow[e] & 0xffff)),
                               bf2f((bf16_t)(vw[e] >> 16)) + bf2f((bf16_t)(ow[e] >> 16)));
          }
          *(uint4*)dst = v;
          if (stats) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float lo = bf2f((bf16_t)(vw[e] & 0xffff)), hi = bf2f((bf16_t)(vw[e] >> 16));
              ssum[2 * e] += lo; ssq[2 * e] += lo * lo;
              ssum[2 * e + 1] += hi; ssq[2 * e + 1] += hi * hi;
            }
          }
        } else {
          for (int e = 0; e < 8 && col + e < N; ++e) {
            float v = bf2f(src[e]);
            if (ep.mask && bf2f(ep.mask[(long)row * ep.ldm + col + e]) <= 0.f) v = 0.f;
            if (ep.mode == 1) v += bf2f(dst[e]);
            const bf16_t o = f2bf(v);
            dst[e] = o;
            if (stats) { const float f = bf2f(o); ssum[e] += f; ssq[e] += f * f; }
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (stats) {
      // lanes of one chunk -> the wave's rows; the two row-waves of a column
      // half through LDS (the slabs are retired); one fp64 atomic per
      // channel and sum into statistics shard (M-tile % BN_SHARDS)
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          ssum[e] += __shfl_xor(ssum[e], o, 64);
          ssq[e] += __shfl_xor(ssq[e], o, 64);
        }
      __syncthreads();
      float* red = (float*)smem;                   // [wr][wc][sum | sq][WC]
      if (lane < CPR) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          red[((wr * 2 + wc) * 2 + 0) * WC + lane * 8 + e] = ssum[e];
          red[((wr * 2 + wc) * 2 + 1) * WC + lane * 8 + e] = ssq[e];
        }
      }
      __syncthreads();
      if (wr == 0) {
        double* sh = ep.stats + (long)((m0 / BM) % BN_SHARDS) * 2 * N;
        for (int e = lane; e < 2 * WC; e += 64) {
          const int q = e / WC, c = e % WC, col = cbase + c;
          if (col < N)
            unsafeAtomicAdd(sh + q * N + col, (double)(red[((0 * 2 + wc) * 2 + q) * WC + c] +
                                                       red[((1 * 2 + wc) * 2 + q) * WC + c]));
        }
      }
    }
    return;
  }

  // ---- fp32 store / accumulate (no atomics): LDS-staged, 16-B row chunks.
  // A rank-k update with tiny K (VGG's classifier weight gradients, K = the
  // batch) is bound by the read-modify-write of C: whole 16-B chunks of
  // consecutive columns per lane instead of the MFMA layout's 4-B stores
  if (ep.c_f32 && (ep.mode == 0 || ep.mode == 1) && !ep.mask && (ep.ldc & 3) == 0 &&
      (((uintptr_t)ep.c) & 15) == 0) {
    constexpr int WR = BM / 2, WC = BN / 2, HR = WR < 32 ? WR : 32, LDF = WC + 4, CPR = WC / 4;
    static_assert(4 * HR * LDF * 4 <= 2 * (A_BYTES + B_BYTES), "fp32 staging exceeds the igemm LDS");
    float* slab = (float*)smem + wid * (HR * LDF);
    if (kt0 >= kt1) __syncthreads();   // (the K loop ends with a barrier otherwise)
    const int cbase = n0 + wc * WC;
    float bv[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = cbase + 16 * j + (lane & 15);
      bv[j] = (add_bias && col < N) ? bf2f(ep.bias[col]) : 0.f;
    }
#pragma unroll
    for (int h = 0; h < WR / HR; ++h) {
#pragma unroll
      for (int ii = 0; ii < HR / 16; ++ii)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[h * (HR / 16) + ii][j][r] * ep.alpha + bv[j];
            if (ep.relu) v = fmaxf(v, 0.f);
            slab[(16 * ii + 4 * (lane >> 4) + r) * LDF + 16 * j + (lane & 15)] = v;
          }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < (HR * CPR + 63) / 64; ++u) {
        const int idx = u * 64 + lane, lr = idx / CPR, ch = idx % CPR;
        const int row = m0 + wr * WR + h * HR + lr, col = cbase + ch * 4;
        if (lr >= HR || row >= M || col >= N) continue;
        float* dst = (float*)ep.c + (long)row * ep.ldc + col;
        const float* src = slab + lr * LDF + ch * 4;
        if (col + 4 <= N) {
          float4 v = *(const float4*)src;
          if (ep.mode == 1) {
            const float4 o = *(const float4*)dst;
            v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
          }
          *(float4*)dst = v;
        } else {
          for (int e = 0; e < 4 && col + e < N; ++e) dst[e] = ep.mode == 1 ? dst[e] + src[e] : src[e];
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    return;
  }

  // ---- epilogue: C/D map of 16x16x32: col = lane&15, row = (lane>>4)*4 + r
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wc * (BN / 2) + 16 * j + (lane & 15);
    if (col >= N) continue;
    const float bv = add_bias ? bf2f(ep.bias[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * (BM / 2) + 16 * i + 4 * (lane >> 4) + r;
        if (row >= M) continue;
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

}  // namespace tam
