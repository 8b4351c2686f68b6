// tiresias_amd — fused (flash-style) attention for head_dim = 64, bf16 I/O.
//
// Layout: token-major [B][S][H][64] with explicit token strides so the packed
// QKV projection output is consumed in place (no permute/contiguous copies).
//
// Forward works on the TRANSPOSED score tile S^T = K Q^T (v_mfma 16x16x32,
// K rows from an LDS image, Q fragments resident in registers): each lane
// then holds 16 scores of ONE query, so the softmax row reductions are 16
// in-lane ops + 2 xor-shuffles, the rescale of O is a per-lane scalar, and
// P^T feeds the O^T += V^T P^T MFMA directly from the accumulator registers
// (k-order permuted; V's LDS rows are stored permuted to match — guide §3
// 'An accumulator tile as the next MFMA's operand').
//
// Backward: one workgroup per (b, h, 64-key block), each wave owns 16 keys
// and keeps dK^T / dV^T in registers across the whole query sweep; S and dP
// are recomputed per 64-query tile (P = exp(S*scale - LSE)), dS crosses LDS
// once (for dQ), dQ is summed across key blocks with fp32 atomics.
#include "tam/common.h"
#include "tam/igemm.h"
#include "tam/kernels.h"

namespace tam {

constexpr int AD = 64;        // head dim
constexpr int AT = 64;        // tile (queries per fwd block / keys per tile)
constexpr float kLog2e = 1.4426950408889634f;

// 32-row-block row permutation for the transposed-read image:
// kv_local = 16h + 4g + q  ->  LDS row 8g + 4h + q
__device__ __forceinline__ int rho(int kv) {
  const int base = kv & ~31, l = kv & 31;
  const int h = l >> 4, g = (l >> 2) & 3, q = l & 3;
  return base + 8 * g + 4 * h + q;
}

// Cooperative 64x64 tile load (256 threads, 2 x 16 B each) from a token-major
// tensor: rows [row0, row0+64), element (r, d) at base + r*stride + d.
__device__ __forceinline__ void tile_fetch(const bf16_t* base, long stride, int row0, int nrows,
                                           uint4 (&r)[2], int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (tid >> 3) + 32 * i, c = tid & 7;
    const int gr = row0 + row;
    r[i] = gr < nrows ? *(const uint4*)(base + (long)gr * stride + 8 * c) : make_uint4(0, 0, 0, 0);
  }
}
// K-major image (row reads by ds_read_b128)
__device__ __forceinline__ void tile_store_k(char* t, const uint4 (&r)[2], int tid, bool perm) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int row = (tid >> 3) + 32 * i;
    if (perm) row = rho(row);
    *(uint4*)(t + kmaj_off(row, tid & 7)) = r[i];
  }
}
// MN-major image (transposed reads by ds_read_b64_tr_b16), optional rho perm
__device__ __forceinline__ void tile_store_mn(char* t, const uint4 (&r)[2], int tid, bool perm) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int row = (tid >> 3) + 32 * i;
    if (perm) row = rho(row);
    *(uint4*)(t + mnmaj_off<64>(row, 2 * (tid & 7))) = r[i];
  }
}

__device__ __forceinline__ s16x8_t pack_frag(const f32x4_t& a, const f32x4_t& b) {
  s16x8_t f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    f[r] = (short)f2bf(a[r]);
    f[4 + r] = (short)f2bf(b[r]);
  }
  return f;
}

__device__ __forceinline__ f32x4_t mfma(const s16x8_t& a, const s16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

// ============================================================== forward
__global__ void __launch_bounds__(256) attn_fwd_kernel(const bf16_t* __restrict__ Q,
                                                        const bf16_t* __restrict__ K,
                                                        const bf16_t* __restrict__ V,
                                                        bf16_t* __restrict__ O,
                                                        float* __restrict__ LSE, int H, int Sq,
                                                        int Sk, long qs, long kvs, long os,
                                                        long qb, long kvb, long ob,
                                                        int causal, float scale,
                                                        const int* __restrict__ kv_len) {
  __shared__ __attribute__((aligned(16))) char smem[2 * AT * AD * 2];
  char* kt = smem;
  char* vt = smem + AT * AD * 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int q0 = blockIdx.x * AT;
  const int qw = q0 + 16 * w + (lane & 15);   // this lane's query
  const int klen = kv_len ? min(Sk, kv_len[b]) : Sk;

  const bf16_t* Qb = Q + (long)b * qb + h * AD;
  const bf16_t* Kb = K + (long)b * kvb + h * AD;
  const bf16_t* Vb = V + (long)b * kvb + h * AD;

  // Q^T fragments as the B operand: lane holds Q[q = lane&15][d = 8g + j + 32ks]
  s16x8_t qf[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    if (qw < Sq) qf[ks] = *(const s16x8_t*)(Qb + (long)qw * qs + 32 * ks + 8 * g);
    else qf[ks] = s16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  const float sl2 = scale * kLog2e;
  float m = -1e30f, l = 0.f;
  f32x4_t o[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) o[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  int kend = klen;
  if (causal) kend = min(kend, q0 + AT);
  // the next K / V tile is fetched into registers right after the current
  // one reaches LDS, so its global latency hides under this tile's math
  uint4 rk[2], rv[2];
  if (kend > 0) {
    tile_fetch(Kb, kvs, 0, klen, rk, tid);
    tile_fetch(Vb, kvs, 0, klen, rv, tid);
  }
  for (int k0 = 0; k0 < kend; k0 += AT) {
    __syncthreads();   // previous tile fully consumed
    tile_store_k(kt, rk, tid, false);
    tile_store_mn(vt, rv, tid, true);
    __syncthreads();
    if (k0 + AT < kend) {
      tile_fetch(Kb, kvs, k0 + AT, klen, rk, tid);
      tile_fetch(Vb, kvs, k0 + AT, klen, rv, tid);
    }
    // S^T[kv][q] : 4 kv sub-tiles x 2 k-steps
    f32x4_t st[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) st[t] = mfma(read_frag_k(kt, lane, 16 * t, ks), qf[ks], st[t]);
    }
    float tmax = -1e30f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kv = k0 + 16 * t + 4 * g + r;
        float v = st[t][r] * sl2;
        if (kv >= klen || (causal && kv > qw)) v = -INFINITY;
        st[t][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax);
    const float alpha = exp2f(m - mn);
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(st[t][r] - mn);
        st[t][r] = p;
        psum += p;
      }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l = l * alpha + psum;
    m = mn;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) o[mt] *= alpha;
    // O^T[d][q] += V^T[d][kv] P^T[kv][q]
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const s16x8_t pb = pack_frag(st[2 * s], st[2 * s + 1]);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        o[mt] = mfma(read_frag_mn<64>(vt, lane, 32 * s, 16 * mt), pb, o[mt]);
    }
  }
  if (qw < Sq) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16_t* Ob = O + (long)b * ob + (long)qw * os + h * AD;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int d = 16 * mt + 4 * g;
      *(uint2*)(Ob + d) = make_uint2(pack_bf2(o[mt][0] * inv, o[mt][1] * inv),
                                     pack_bf2(o[mt][2] * inv, o[mt][3] * inv));
    }
    if (g == 0 && LSE)
      LSE[((long)b * H + h) * Sq + qw] = l > 0.f ? (m + __log2f(l)) * 0.6931471805599453f : -INFINITY;
  }
}

// delta[b,h,q] = sum_d dO * O, and the same wave zeroes that row's fp32 dQ
// accumulator ([B][Sq][H][64]) -- one launch instead of delta + a memset
__global__ void attn_delta_kernel(const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO,
                                  float* __restrict__ delta, float* __restrict__ dq_acc, int B,
                                  int H, int Sq, long os, long ob) {
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= (long)B * H * Sq) return;
  const int q = (int)(row % Sq);
  const long bh = row / Sq;
  const int h = (int)(bh % H), b = (int)(bh / H);
  const long off = (long)b * ob + (long)q * os + h * AD + lane;
  dq_acc[(((long)b * Sq + q) * H + h) * AD + lane] = 0.f;
  float v = bf2f(O[off]) * bf2f(dO[off]);
  v = wave_sum(v);
  if (lane == 0) delta[row] = v;
}

// ============================================================== backward
__global__ void __launch_bounds__(256) attn_bwd_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
    bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, float* __restrict__ dQacc, int H, int Sq,
    int Sk, long qs, long kvs, long os, long qb, long kvb, long ob, int causal, float scale,
    const int* __restrict__ kv_len) {
  // LDS: Q row image, Q^T image (rho), dO row image, dO^T image (rho), K^T image, dS image,
  //      lse[64], delta[64]
  __shared__ __attribute__((aligned(16))) char smem[6 * AT * AD * 2 + 2 * AT * 4];
  char* q_k = smem;
  char* q_mn = smem + 1 * AT * AD * 2;
  char* do_k = smem + 2 * AT * AD * 2;
  char* do_mn = smem + 3 * AT * AD * 2;
  char* k_mn = smem + 4 * AT * AD * 2;
  char* ds_mn = smem + 5 * AT * AD * 2;
  float* s_lse = (float*)(smem + 6 * AT * AD * 2);
  float* s_del = s_lse + AT;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int k0 = blockIdx.x * AT;
  const int klen = kv_len ? min(Sk, kv_len[b]) : Sk;
  const int kvw = k0 + 16 * w + (lane & 15);   // this lane's key (column of S)

  const bf16_t* Qb = Q + (long)b * qb + h * AD;
  const bf16_t* dOb = dO + (long)b * ob + h * AD;
  const bf16_t* Kb = K + (long)b * kvb + h * AD;
  const bf16_t* Vb = V + (long)b * kvb + h * AD;
  const float* lse_b = LSE + ((long)b * H + h) * Sq;
  const float* del_b = DELTA + ((long)b * H + h) * Sq;

  // K, V fragments of this wave's 16 keys as B operands (n = key, k = d)
  s16x8_t kf[2], vf[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const bool ok = kvw < klen;
    kf[ks] = ok ? *(const s16x8_t*)(Kb + (long)kvw * kvs + 32 * ks + 8 * g) : s16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    vf[ks] = ok ? *(const s16x8_t*)(Vb + (long)kvw * kvs + 32 * ks + 8 * g) : s16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  {  // K image [kv][d] for dQ = dS K (B operand, k = kv, n = d: MN-major)
    uint4 rk[2];
    tile_fetch(Kb, kvs, k0, klen, rk, tid);
    tile_store_mn(k_mn, rk, tid, false);
  }
  f32x4_t dvt[4], dkt[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) dvt[mt] = dkt[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const float sl2 = scale * kLog2e;

  const int qstart = causal ? (k0 / AT) * AT : 0;
  for (int q0 = qstart; q0 < Sq; q0 += AT) {
    uint4 rq[2], rd[2];
    tile_fetch(Qb, qs, q0, Sq, rq, tid);
    tile_fetch(dOb, os, q0, Sq, rd, tid);
    __syncthreads();   // previous iteration done with all images
    tile_store_k(q_k, rq, tid, false);
    tile_store_mn(q_mn, rq, tid, true);
    tile_store_k(do_k, rd, tid, false);
    tile_store_mn(do_mn, rd, tid, true);
    if (tid < AT) {
      const int q = q0 + tid;
      s_lse[tid] = q < Sq ? lse_b[q] * kLog2e : 0.f;
      s_del[tid] = q < Sq ? del_b[q] : 0.f;
    }
    __syncthreads();
    // S[q][kv] and dP[q][kv]: 4 q sub-tiles (t) x 2 k-steps; row q = 16t + 4g + r, col kv = lane&15
    f32x4_t sp[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sp[t] = dp[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        sp[t] = mfma(read_frag_k(q_k, lane, 16 * t, ks), kf[ks], sp[t]);
        dp[t] = mfma(read_frag_k(do_k, lane, 16 * t, ks), vf[ks], dp[t]);
      }
    }
    // P = exp2(S*scale*log2e - lse*log2e); dS = P * (dP - delta)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * t + 4 * g + r;
        const int q = q0 + ql;
        float p = exp2f(sp[t][r] * sl2 - s_lse[ql]);
        if (q >= Sq || kvw >= klen || (causal && kvw > q)) p = 0.f;
        sp[t][r] = p;
        dp[t][r] = p * (dp[t][r] - s_del[ql]);
      }
    // dV^T[d][kv] += dO^T[d][q] P[q][kv] ; dK^T[d][kv] += Q^T[d][q] dS[q][kv]
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const s16x8_t pb = pack_frag(sp[2 * s], sp[2 * s + 1]);
      const s16x8_t sb = pack_frag(dp[2 * s], dp[2 * s + 1]);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        dvt[mt] = mfma(read_frag_mn<64>(do_mn, lane, 32 * s, 16 * mt), pb, dvt[mt]);
        dkt[mt] = mfma(read_frag_mn<64>(q_mn, lane, 32 * s, 16 * mt), sb, dkt[mt]);
      }
    }
    // dS -> LDS as [kv][q] (MN-major for the dQ A operand: m = q, k = kv)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int kvl = 16 * w + (lane & 15);
      const int c8 = (16 * t + 4 * g) >> 2;
      *(uint2*)(ds_mn + mnmaj_off<64>(kvl, c8)) =
          make_uint2(pack_bf2(dp[t][0], dp[t][1]), pack_bf2(dp[t][2], dp[t][3]));
    }
    __syncthreads();
    // dQ[q][d] (this wave: q rows 16w..16w+15) = dS[q][kv] K[kv][d] over the block's 64 keys
    f32x4_t dq[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dq[nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const s16x8_t a = read_frag_mn<64>(ds_mn, lane, 32 * s, 16 * w);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dq[nt] = mfma(a, read_frag_mn<64>(k_mn, lane, 32 * s, 16 * nt), dq[nt]);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = q0 + 16 * w + 4 * g + r;
        if (q < Sq) {
          const int d = 16 * nt + (lane & 15);
          atomicAdd(dQacc + ((long)b * Sq + q) * (long)(H * AD) + h * AD + d, dq[nt][r] * scale);
        }
      }
  }
  if (kvw < Sk) {
    bf16_t* dKb = dK + (long)b * kvb + (long)kvw * kvs + h * AD;
    bf16_t* dVb = dV + (long)b * kvb + (long)kvw * kvs + h * AD;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int d = 16 * mt + 4 * g;
      *(uint2*)(dKb + d) = make_uint2(pack_bf2(dkt[mt][0] * scale, dkt[mt][1] * scale),
                                      pack_bf2(dkt[mt][2] * scale, dkt[mt][3] * scale));
      *(uint2*)(dVb + d) = make_uint2(pack_bf2(dvt[mt][0], dvt[mt][1]), pack_bf2(dvt[mt][2], dvt[mt][3]));
    }
  }
}

// ============================================================== backward, Sk <= 128
// Short key ranges (the Transformer's 128-token sequences): ONE workgroup of
// 8 waves per (b, h) owns every key (waves 0-3: keys 0-63, 4-7: keys 64-127,
// 16 per wave, dK^T / dV^T in registers as in attn_bwd_kernel) and sweeps the
// query tiles. With all keys in the block, a query tile's dQ = dS K over the
// 128 keys is finished in-block (dS [kv][q] and K [kv][d] LDS images) and
// stored as bf16 directly; delta = rowsum(dO * O) is formed in-block from the
// dO and O tile images. One launch instead of delta+zero / backward /
// fp32-dQ cast, and no dQ atomics.
constexpr int ATS_K = 128;
__global__ void __launch_bounds__(512) attn_bwd_short_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO, const float* __restrict__ LSE,
    bf16_t* __restrict__ dQ, bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int H, int Sq, int Sk,
    long qs, long kvs, long os, long qb, long kvb, long ob, int causal, float scale,
    const int* __restrict__ kv_len) {
  // LDS: Q row image, Q^T image (rho), dO row image, dO^T image (rho), O row
  //      image (delta), K [kv][d] image (128 rows), dS [kv][q] image (128 rows),
  //      lse[64], delta[64]
  constexpr int T = AT * AD * 2;     // one 64x64 bf16 image
  __shared__ __attribute__((aligned(16))) char smem[5 * T + 2 * 2 * T + 2 * AT * 4];
  char* q_k = smem;
  char* q_mn = smem + 1 * T;
  char* do_k = smem + 2 * T;
  char* do_mn = smem + 3 * T;
  char* o_k = smem + 4 * T;
  char* k_mn = smem + 5 * T;          // [128 kv][64 d]
  char* ds_mn = smem + 7 * T;         // [128 kv][64 q]
  float* s_lse = (float*)(smem + 9 * T);
  float* s_del = s_lse + AT;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int half = tid >> 8, ht = tid & 255;          // 256-thread halves
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int klen = kv_len ? min(Sk, kv_len[b]) : Sk;
  const int kvw = 16 * w + (lane & 15);               // this lane's key (0..127)

  const bf16_t* Qb = Q + (long)b * qb + h * AD;
  const bf16_t* dOb = dO + (long)b * ob + h * AD;
  const bf16_t* Ob = O + (long)b * ob + h * AD;
  const bf16_t* Kb = K + (long)b * kvb + h * AD;
  const bf16_t* Vb = V + (long)b * kvb + h * AD;
  const float* lse_b = LSE + ((long)b * H + h) * Sq;

  // query tile q0's Q (half 0) / dO, O (half 1) rows and LSE, fetched into
  // registers one tile AHEAD: the first with the K / V loads below, the next
  // right after the current one reaches LDS (its latency hides under the math)
  uint4 ra[2], rb[2];
  float lse_r = 0.f;
  auto fetch_q = [&](int q0) {
    if (half == 0) {
      tile_fetch(Qb, qs, q0, Sq, ra, ht);
      if (ht < AT) lse_r = q0 + ht < Sq ? lse_b[q0 + ht] : 0.f;
    } else {
      tile_fetch(dOb, os, q0, Sq, ra, ht);
      tile_fetch(Ob, os, q0, Sq, rb, ht);
    }
  };
  if (Sq > 0) fetch_q(0);
  s16x8_t kf[2], vf[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const bool ok = kvw < klen;
    kf[ks] = ok ? *(const s16x8_t*)(Kb + (long)kvw * kvs + 32 * ks + 8 * g) : s16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    vf[ks] = ok ? *(const s16x8_t*)(Vb + (long)kvw * kvs + 32 * ks + 8 * g) : s16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  {  // K image: half 0 keys 0-63, half 1 keys 64-127 (rows 64*half + r)
    uint4 rk[2];
    tile_fetch(Kb, kvs, 64 * half, klen, rk, ht);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 64 * half + (ht >> 3) + 32 * i;
      *(uint4*)(k_mn + mnmaj_off<64>(row, 2 * (ht & 7))) = rk[i];
    }
  }
  f32x4_t dvt[4], dkt[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) dvt[mt] = dkt[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const float sl2 = scale * kLog2e;

  for (int q0 = 0; q0 < Sq; q0 += AT) {
    // half 0 stages Q, half 1 stages dO and O (fetched one tile ahead)
    __syncthreads();   // previous iteration done with all images
    if (half == 0) {
      tile_store_k(q_k, ra, ht, false);
      tile_store_mn(q_mn, ra, ht, true);
      if (ht < AT) s_lse[ht] = lse_r * kLog2e;
    } else {
      tile_store_k(do_k, ra, ht, false);
      tile_store_mn(do_mn, ra, ht, true);
      tile_store_k(o_k, rb, ht, false);
    }
    __syncthreads();
    if (q0 + AT < Sq) fetch_q(q0 + AT);
    {  // delta[q] = sum_d dO[q][d] O[q][d]: 8 threads per row, 8 d each
      const int row = tid >> 3, c = tid & 7;
      const uint4 a = *(const uint4*)(do_k + kmaj_off(row, c));
      const uint4 o = *(const uint4*)(o_k + kmaj_off(row, c));
      const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, ow[4] = {o.x, o.y, o.z, o.w};
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        d += __uint_as_float(aw[e] << 16) * __uint_as_float(ow[e] << 16);
        d += __uint_as_float(aw[e] & 0xffff0000u) * __uint_as_float(ow[e] & 0xffff0000u);
      }
      d += __shfl_xor(d, 1, 64);
      d += __shfl_xor(d, 2, 64);
      d += __shfl_xor(d, 4, 64);
      if (c == 0) s_del[row] = d;
    }
    __syncthreads();
    // S[q][kv], dP[q][kv] for this wave's 16 keys: q = 16t + 4g + r
    f32x4_t sp[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sp[t] = dp[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        sp[t] = mfma(read_frag_k(q_k, lane, 16 * t, ks), kf[ks], sp[t]);
        dp[t] = mfma(read_frag_k(do_k, lane, 16 * t, ks), vf[ks], dp[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * t + 4 * g + r;
        const int q = q0 + ql;
        float p = exp2f(sp[t][r] * sl2 - s_lse[ql]);
        if (q >= Sq || kvw >= klen || (causal && kvw > q)) p = 0.f;
        sp[t][r] = p;
        dp[t][r] = p * (dp[t][r] - s_del[ql]);
      }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const s16x8_t pb = pack_frag(sp[2 * s], sp[2 * s + 1]);
      const s16x8_t sb = pack_frag(dp[2 * s], dp[2 * s + 1]);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        dvt[mt] = mfma(read_frag_mn<64>(do_mn, lane, 32 * s, 16 * mt), pb, dvt[mt]);
        dkt[mt] = mfma(read_frag_mn<64>(q_mn, lane, 32 * s, 16 * mt), sb, dkt[mt]);
      }
    }
    // dS -> LDS [kv][q]
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c8 = (16 * t + 4 * g) >> 2;
      *(uint2*)(ds_mn + mnmaj_off<64>(kvw, c8)) =
          make_uint2(pack_bf2(dp[t][0], dp[t][1]), pack_bf2(dp[t][2], dp[t][3]));
    }
    __syncthreads();
    // dQ[q][d] over all 128 keys: wave w -> q rows 16*(w&3), d columns 32*(w>>2) + {0, 16}
    f32x4_t dq[2];
    dq[0] = dq[1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < ATS_K / 32; ++s) {
      const s16x8_t a = read_frag_mn<64>(ds_mn, lane, 32 * s, 16 * (w & 3));
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        dq[nt] = mfma(a, read_frag_mn<64>(k_mn, lane, 32 * s, 32 * (w >> 2) + 16 * nt), dq[nt]);
    }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = q0 + 16 * (w & 3) + 4 * g + r;
        if (q < Sq) {
          const int d = 32 * (w >> 2) + 16 * nt + (lane & 15);
          dQ[(long)b * qb + (long)q * qs + h * AD + d] = f2bf(dq[nt][r] * scale);
        }
      }
  }
  if (kvw < Sk) {
    bf16_t* dKb = dK + (long)b * kvb + (long)kvw * kvs + h * AD;
    bf16_t* dVb = dV + (long)b * kvb + (long)kvw * kvs + h * AD;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int d = 16 * mt + 4 * g;
      *(uint2*)(dKb + d) = make_uint2(pack_bf2(dkt[mt][0] * scale, dkt[mt][1] * scale),
                                      pack_bf2(dkt[mt][2] * scale, dkt[mt][3] * scale));
      *(uint2*)(dVb + d) = make_uint2(pack_bf2(dvt[mt][0], dvt[mt][1]), pack_bf2(dvt[mt][2], dvt[mt][3]));
    }
  }
}

// dq (bf16, strided like Q) = dq_acc (fp32, packed [B][Sq][H][64])
__global__ void attn_dq_cast_kernel(const float* __restrict__ acc, bf16_t* __restrict__ dq, long n,
                                    int HD, int Sq, long qs, long qb) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long tok = i / HD;
    const int c = (int)(i % HD);
    dq[(tok / Sq) * qb + (tok % Sq) * qs + c] = f2bf(acc[i]);
  }
}

void attn_forward(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B,
                  int H, int Sq, int Sk, long q_stride, long kv_stride, long o_stride, long q_bstride,
                  long kv_bstride, long o_bstride, int causal, float scale, const int* kv_len, hipStream_t s) {
  dim3 grid((Sq + AT - 1) / AT, B * H);
  hipLaunchKernelGGL(attn_fwd_kernel, grid, dim3(256), 0, s, q, k, v, o, lse, H, Sq, Sk, q_stride,
                     kv_stride, o_stride, q_bstride, kv_bstride, o_bstride, causal, scale, kv_len);
}

// 1 (default): key ranges <= 128 take the one-launch short-sequence backward;
// 0: always the key-blocked kernels (tests / A/B)
static int g_attn_short = 1;
TAM_KNOB(g_attn_short)
void attn_short_policy(int p) { g_attn_short = p; }

void attn_backward(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o,
                   const bf16_t* dout, const float* lse, bf16_t* dq, bf16_t* dk, bf16_t* dv,
                   float* dq_acc, float* delta, int B, int H, int Sq, int Sk, long q_stride,
                   long kv_stride, long o_stride, long q_bstride, long kv_bstride, long o_bstride, int causal,
                   float scale, const int* kv_len, hipStream_t s) {
  if (Sk <= ATS_K && g_attn_short) {
    hipLaunchKernelGGL(attn_bwd_short_kernel, dim3(B * H), dim3(512), 0, s, q, k, v, o, dout, lse, dq, dk, dv,
                       H, Sq, Sk, q_stride, kv_stride, o_stride, q_bstride, kv_bstride, o_bstride, causal, scale,
                       kv_len);
    return;
  }
  const long rows = (long)B * H * Sq;
  hipLaunchKernelGGL(attn_delta_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, o, dout, delta, dq_acc,
                     B, H, Sq, o_stride, o_bstride);
  const long nq = (long)B * Sq * H * AD;
  dim3 grid((Sk + AT - 1) / AT, B * H);
  hipLaunchKernelGGL(attn_bwd_kernel, grid, dim3(256), 0, s, q, k, v, dout, lse, delta, dk, dv,
                     dq_acc, H, Sq, Sk, q_stride, kv_stride, o_stride, q_bstride, kv_bstride, o_bstride, causal,
                     scale, kv_len);
  long blocks = (nq + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(attn_dq_cast_kernel, dim3(blocks), dim3(256), 0, s, dq_acc, dq, nq, H * AD, Sq,
                     q_stride, q_bstride);
}

}  // namespace tam
