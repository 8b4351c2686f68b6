// tiresias_amd — BatchNorm (NHWC, training) and LayerNorm kernels.
//
// BatchNorm is split into a stats pass (per-channel sum / sum-of-squares,
// fp32 per block -> fp64 atomics, skipped when the producing conv's epilogue
// already accumulated them) and a fused apply pass (per-channel finalize in
// its prologue, then scale/shift + optional residual add + optional ReLU, 16 B
// per lane). Backward mirrors it: one reduction pass (or the consumer conv's
// dgrad epilogue) accumulating sum(d), sum(d*xhat), and one fused pass
// producing dx (and the residual-branch gradient) plus dgamma/dbeta.
#include "tam/common.h"
#include "tam/kernels.h"

namespace tam {

__device__ __forceinline__ void unpack8(const uint4 v, float (&f)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]),
                    pack_bf2(f[6], f[7]));
}

// ---------------------------------------------------------------- column reduce
// Second stage of every atomic-free reduction here: out[c] = sum_b part[b][c]
// over nblk partial rows of width W, in fp64. Block = 16 columns x 16 row
// lanes (64 B coalesced segments), 8 independent loads in flight per lane so
// the pass is not a serial chain of HBM round trips.
template <int MODE>   // 0: fp64 store to out64; 1: fp32 accumulate into out0[c<split] / out1[c-split]
__global__ void __launch_bounds__(256) col_reduce_kernel(const float* __restrict__ part, int nblk,
                                                          int W, double* __restrict__ out64,
                                                          float* __restrict__ out0,
                                                          float* __restrict__ out1, int split) {
  __shared__ double red[16][17];
  const int cx = threadIdx.x & 15, ly = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cx;
  double s = 0.0;
  if (c < W) {
    int b = ly;
    for (; b + 7 * 16 < nblk; b += 8 * 16) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(long)(b + u * 16) * W + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += (double)v[u];
    }
    for (; b < nblk; b += 16) s += (double)part[(long)b * W + c];
  }
  red[ly][cx] = s;
  __syncthreads();
  if (ly == 0 && c < W) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][cx];
    if (MODE == 0) out64[c] = t;
    else if (c < split) out0[c] += (float)t;
    else out1[c - split] += (float)t;
  }
}

// Many column reduces in ONE launch (the deferred LayerNorm weight-gradient
// reductions of a backward, ops/functional.py flush_wgrad): blocks
// [c0_e, c0_{e+1}) serve entry e, 16 columns each, exactly as
// col_reduce_kernel<1> would for that entry alone.
struct ColRedBatch {
  const float* part[CR_BATCH_MAX];
  float* out0[CR_BATCH_MAX];
  float* out1[CR_BATCH_MAX];
  int nblk[CR_BATCH_MAX], W[CR_BATCH_MAX], split[CR_BATCH_MAX], c0[CR_BATCH_MAX + 1];
  int n;
};

__global__ void __launch_bounds__(256) col_reduce_batch_kernel(ColRedBatch b) {
  __shared__ double red[16][17];
  int e = 0;
  while (e + 1 < b.n && (int)blockIdx.x >= b.c0[e + 1]) ++e;
  const float* __restrict__ part = b.part[e];
  const int nblk = b.nblk[e], W = b.W[e], split = b.split[e];
  const int cx = threadIdx.x & 15, ly = threadIdx.x >> 4;
  const int c = ((int)blockIdx.x - b.c0[e]) * 16 + cx;
  double s = 0.0;
  if (c < W) {
    int k = ly;
    for (; k + 7 * 16 < nblk; k += 8 * 16) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(long)(k + u * 16) * W + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += (double)v[u];
    }
    for (; k < nblk; k += 16) s += (double)part[(long)k * W + c];
  }
  red[ly][cx] = s;
  __syncthreads();
  if (ly == 0 && c < W) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][cx];
    if (c < split) b.out0[e][c] += (float)t;
    else b.out1[e][c - split] += (float)t;
  }
}

void col_reduce_acc_batch(const float* const* part, const int* nblk, const int* W, float* const* out0,
                          float* const* out1, const int* split, int n, hipStream_t s) {
  for (int base = 0; base < n; base += CR_BATCH_MAX) {
    ColRedBatch b{};
    const int m = n - base < CR_BATCH_MAX ? n - base : CR_BATCH_MAX;
    int blocks = 0;
    for (int i = 0; i < m; ++i) {
      b.part[i] = part[base + i]; b.out0[i] = out0[base + i]; b.out1[i] = out1[base + i];
      b.nblk[i] = nblk[base + i]; b.W[i] = W[base + i]; b.split[i] = split[base + i];
      b.c0[i] = blocks;
      blocks += (W[base + i] + 15) / 16;
    }
    b.c0[m] = blocks;
    b.n = m;
    if (blocks) hipLaunchKernelGGL(col_reduce_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, s, b);
  }
}

void col_reduce_f64(const float* part, int nblk, int W, double* out, hipStream_t s) {
  hipLaunchKernelGGL(col_reduce_kernel<0>, dim3((W + 15) / 16), dim3(256), 0, s, part, nblk, W, out,
                     (float*)nullptr, (float*)nullptr, W);
}
void col_reduce_acc(const float* part, int nblk, int W, float* out0, float* out1, int split,
                    hipStream_t s) {
  hipLaunchKernelGGL(col_reduce_kernel<1>, dim3((W + 15) / 16), dim3(256), 0, s, part, nblk, W,
                     (double*)nullptr, out0, out1, split);
}

// ---------------------------------------------------------------- BN sums
// Per-channel statistics live in fp64 sums[BN_SHARDS][2C] (sum | sum of
// squares, or sum(d) | sum(d*xhat) in backward); a channel's value is the sum
// over the shards, taken by the consumer's prologue, which derives mean/rstd
// (or the backward coefficients) itself -- there is no finalize launch.
//   * conv epilogues (conv_dma.h, Epi::stats) add each M-tile's column sums
//     with no-return device-scope atomics into shard tm % BN_SHARDS: tiles
//     finish spread over the conv, and the shards keep the adders per address
//     low (same-address fp64 atomics serialise at the memory side: 512
//     simultaneous adders per address measured +85 us on a 13 us pass);
//   * this file's reduction passes (<= BN_MAX_BLOCKS blocks) add each
//     block's column sums the same way into shard blockIdx % BN_SHARDS
//     (<= 32 adders per address; no partial rows, no column-reduce launch).
// fp64 keeps E[x^2] - E[x]^2 from cancelling at N*H*W ~ 10^5-10^6. The
// caller zeroes sums beforehand (one fill per training step for all of a
// model's BNs).

constexpr int BN_SLAB = 256;

// a channel's (S, Q) over the shards
__device__ __forceinline__ void bn_shard_sum(const double* __restrict__ sums, int C, int c, double& S,
                                             double& Q) {
  double s[BN_SHARDS], q[BN_SHARDS];
#pragma unroll
  for (int k = 0; k < BN_SHARDS; ++k) {
    s[k] = sums[(long)k * 2 * C + c];
    q[k] = sums[(long)k * 2 * C + C + c];
  }
  S = 0.0; Q = 0.0;
#pragma unroll
  for (int k = 0; k < BN_SHARDS; ++k) { S += s[k]; Q += q[k]; }
}

// a reducing block's 2C column sums (held by its row-lane-0 threads, 8
// channels each) -> LDS -> no-return fp64 atomics into shard blockIdx %
// BN_SHARDS (<= 32 adders per address at BN_MAX_BLOCKS blocks), issued by
// every thread over CONTIGUOUS addresses (512 B per wave instruction; the
// per-thread 8-channel strided form measured 1.75x slower on ResNet-50's
// backward reductions)
__device__ __forceinline__ void bn_block_atomics(float* red, const float (&s)[8], const float (&q)[8], bool owner,
                                                 int cg, int cs, int c0, int C, double* __restrict__ sums) {
  __syncthreads();                       // red's partial rows are consumed
  if (owner) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { red[cg * 8 + i] = s[i]; red[cs + cg * 8 + i] = q[i]; }
  }
  __syncthreads();
  double* sh = sums + (long)(blockIdx.x % BN_SHARDS) * 2 * C + c0;
  for (int e = threadIdx.x; e < 2 * cs; e += blockDim.x) {
    const int hi = e >= cs;
    unsafeAtomicAdd(sh + hi * C + (e - hi * cs), (double)red[e]);
  }
}

// Reduction passes run over a 2-D grid: blockIdx.y = a slab of <= sw
// channels (sw = BN_SLAB, or C itself with g_bn_red_slab = 0), blockIdx.x a
// contiguous row range. Each block adds 2 * sw fp64 atomics, so slabbing a
// wide BN (C = 1024 / 2048 on ResNet-50's 14x14 / 7x7 layers) lets each block
// cover more rows for the same grid: the full-width form issued 1-1.8 M
// atomics per pass there against 262 K now.
static int g_bn_red_slab = [] {
  const char* e = getenv("TAM_BN_RED_SLAB");
  return e ? atoi(e) : 1;
}();
TAM_KNOB(g_bn_red_slab)
static int g_bn_red_blocks = [] {
  const char* e = getenv("TAM_BN_RED_BLOCKS");
  return e ? atoi(e) : BN_MAX_BLOCKS;
}();
TAM_KNOB(g_bn_red_blocks)

struct BnRed {
  dim3 grid;
  long rows_per_block;
  int sw;
};

static BnRed bn_reduce_grid(long M, int C) {
  const int sw = g_bn_red_slab && C > BN_SLAB ? BN_SLAB : C;
  const int slabs = (C + sw - 1) / sw;
  const int nbmax = g_bn_red_blocks > 0 ? g_bn_red_blocks : BN_MAX_BLOCKS;
  long rx = nbmax / slabs;
  if (rx < 1) rx = 1;
  // each block streams >= 4 passes of its thread grid so the loads stay 16 B/lane
  long rpb = (M + rx - 1) / rx;
  const long minr = 256 / (sw / 8) * 4;
  if (rpb < minr) rpb = minr;
  return BnRed{dim3((unsigned)((M + rpb - 1) / rpb), (unsigned)slabs), rpb, sw};
}

// grid.x blocks each own a contiguous row range; thread = (row lane, 8-ch group)
__global__ void __launch_bounds__(256) bn_stats_kernel(const bf16_t* __restrict__ x, long M, int C,
                                                        long rows_per_block, int sw,
                                                        double* __restrict__ sums) {
  __shared__ float red[256 * 16];
  const int c0 = blockIdx.y * sw;
  const int cs = min(sw, C - c0);
  const int tpr = cs / 8;                // threads per row
  const int rpb = 256 / tpr;             // rows per pass (cs <= 2048)
  const int cg = threadIdx.x % tpr, rl = threadIdx.x / tpr;
  x += c0;
  float s[8], q[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = q[i] = 0.f;
  const long r0 = blockIdx.x * rows_per_block;
  const long r1 = min(M, r0 + rows_per_block);
  if (rl < rpb) {
    long r = r0 + rl;
    // 4 independent 16-B loads in flight per thread (latency, not bandwidth,
    // bounds a one-load-per-iteration loop)
    for (; r + 3 * rpb < r1; r += 4 * rpb) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *(const uint4*)(x + (r + u * rpb) * C + cg * 8);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int i = 0; i < 8; ++i) { s[i] += f[i]; q[i] += f[i] * f[i]; }
      }
    }
    for (; r < r1; r += rpb) {
      float f[8];
      unpack8(*(const uint4*)(x + r * C + cg * 8), f);
#pragma unroll
      for (int i = 0; i < 8; ++i) { s[i] += f[i]; q[i] += f[i] * f[i]; }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[threadIdx.x * 16 + i] = s[i]; red[threadIdx.x * 16 + 8 + i] = q[i]; }
  __syncthreads();
  if (rl == 0) {
    for (int j = 1; j < rpb; ++j) {
      const int t = j * tpr + cg;
#pragma unroll
      for (int i = 0; i < 8; ++i) { s[i] += red[t * 16 + i]; q[i] += red[t * 16 + 8 + i]; }
    }
  }
  bn_block_atomics(red, s, q, rl == 0, cg, cs, c0, C, sums);
}

// Apply passes run over a 2-D grid: blockIdx.y = a slab of <= BN_SLAB
// channels, blockIdx.x = a contiguous row range. Each block first derives its
// slab's per-channel coefficients from the fp64 sums into LDS (the old
// finalize kernel, replicated per block: 2 doubles + 2 floats per channel,
// L2-resident), then streams rows with 16 B per lane, 2 rows in flight.
struct BnGrid {
  dim3 grid;
  long rows_per_block;
};

// g_bn_apply_blocks: the grid's block target; 0 (default) = 1024 blocks for
// tensors of >= 32 M elements, 512 below. Each block also reads its slab's 16
// statistics shards (64 KB at 256 channels) from L2, so fewer, longer blocks
// pay: ResNet-50's 53 BN layers, forward + backward apply, 2802 -> 2683 us
// against a flat 2048 (tools/bench_bn.py, same box; flat 1024: 2735, flat
// 512: 2710 -- the 51 M-element stage-1 / stem tensors prefer 1024)
static int g_bn_apply_blocks = [] {
  const char* e = getenv("TAM_BN_APPLY_BLOCKS");
  return e ? atoi(e) : 0;
}();
TAM_KNOB(g_bn_apply_blocks)

static BnGrid bn_apply_grid(long M, int C) {
  const int slabs = (C + BN_SLAB - 1) / BN_SLAB;
  const int vs = (C < BN_SLAB ? C : BN_SLAB) / 8;
  const long rpp = 256 / vs;                              // rows per pass
  const long target = g_bn_apply_blocks > 0 ? g_bn_apply_blocks : (M * C >= (32L << 20) ? 1024 : 512);
  long bx = (target + slabs - 1) / slabs;
  long rpb = (M + bx - 1) / bx;
  if (rpb < 2 * rpp) rpb = 2 * rpp;
  rpb = (rpb + rpp - 1) / rpp * rpp;
  bx = (M + rpb - 1) / rpb;
  return BnGrid{dim3((unsigned)bx, (unsigned)slabs), rpb};
}

// y = x*scale + shift (+res) (relu); scale/shift from the sums. Blocks of row
// range 0 also write save_mean / save_rstd and update the running statistics.
__global__ void __launch_bounds__(256) bn_apply_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ res, bf16_t* __restrict__ y, long M,
    int C, long rows_per_block, const double* __restrict__ sums, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float momentum, float* __restrict__ save_mean,
    float* __restrict__ save_rstd, float* __restrict__ run_mean, float* __restrict__ run_var,
    int relu, uint8_t* __restrict__ ymask) {
  __shared__ float s_sc[BN_SLAB], s_sh[BN_SLAB];
  const int c0 = blockIdx.y * BN_SLAB;
  const int cs = min(BN_SLAB, C - c0);
  const int t = threadIdx.x;
  if (t < cs) {
    const int c = c0 + t;
    double S, Q;
    bn_shard_sum(sums, C, c, S, Q);
    const double mean = S / (double)M;
    double var = Q / (double)M - mean * mean;
    if (var < 0) var = 0;
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = gamma[c] * rstd;
    s_sc[t] = sc;
    s_sh[t] = beta[c] - (float)mean * sc;
    if (blockIdx.x == 0) {
      save_mean[c] = (float)mean;
      save_rstd[c] = rstd;
      if (run_mean) {
        const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
        run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
        run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unb;
      }
    }
  }
  __syncthreads();
  const int vs = cs / 8, rpp = 256 / vs;
  const int v = t % vs, rl = t / vs;
  if (rl >= rpp) return;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = s_sc[v * 8 + j]; sh[j] = s_sh[v * 8 + j]; }
  auto one = [&](const long off, const uint4 vx, const uint4 vr) {
    float f[8], rr[8];
    unpack8(vx, f);
    if (res) unpack8(vr, rr);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float o = f[j] * sc[j] + sh[j];
      if (res) o += rr[j];
      if (relu) o = fmaxf(o, 0.f);
      f[j] = o;
    }
    const uint4 pk = pack8(f);
    *(uint4*)(y + off) = pk;
    if (ymask) {
      // bit j of byte off/8: the STORED bf16 of channel col+j is > 0 (what a
      // ReLU backward reading y would test)
      const uint32_t w[4] = {pk.x, pk.y, pk.z, pk.w};
      uint32_t bits = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bits |= (((w[e] & 0x8000u) == 0 && (w[e] & 0x7fffu) != 0) ? 1u : 0u) << (2 * e);
        bits |= (((w[e] & 0x80000000u) == 0 && (w[e] & 0x7fff0000u) != 0) ? 1u : 0u) << (2 * e + 1);
      }
      ymask[off >> 3] = (uint8_t)bits;
    }
  };
  const uint4 z = make_uint4(0, 0, 0, 0);
  const long r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  const long col = c0 + v * 8;
  long r = r0 + rl;
  for (; r + rpp < r1; r += 2 * rpp) {
    const long o0 = r * C + col, o1 = (r + rpp) * C + col;
    const uint4 x0 = *(const uint4*)(x + o0), x1 = *(const uint4*)(x + o1);
    const uint4 q0 = res ? *(const uint4*)(res + o0) : z, q1 = res ? *(const uint4*)(res + o1) : z;
    one(o0, x0, q0);
    one(o1, x1, q1);
  }
  if (r < r1) {
    const long o0 = r * C + col;
    one(o0, *(const uint4*)(x + o0), res ? *(const uint4*)(res + o0) : z);
  }
}

// ---------------------------------------------------------------- BN backward
// dyr = (dy + addend) * (y > 0 if relu); accum sum(dyr), sum(dyr * xhat) per
// channel (sharded fp64 atomics). dp_out (residual BNs): dyr is also stored -- it IS the
// residual branch's gradient, and the apply pass then reads dyr + x only (no
// dy, addend, y re-reads, no second dres write: 2 passes of the tensor saved)
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ addend, const bf16_t* __restrict__ y,
    const bf16_t* __restrict__ x, const float* __restrict__ mean, const float* __restrict__ rstd, long M,
    int C, long rows_per_block, int sw, int relu, double* __restrict__ sums, bf16_t* __restrict__ dp_out,
    const uint8_t* __restrict__ ymask) {
  __shared__ float red[256 * 16];
  const int c0 = blockIdx.y * sw;
  const int cs = min(sw, C - c0);
  const int tpr = cs / 8, rpb = 256 / tpr;
  const int cg = threadIdx.x % tpr, rl = threadIdx.x / tpr;
  float a[8], b[8], mu[8], rs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { a[i] = b[i] = 0.f; mu[i] = mean[c0 + cg * 8 + i]; rs[i] = rstd[c0 + cg * 8 + i]; }
  const long r0 = blockIdx.x * rows_per_block;
  const long r1 = min(M, r0 + rows_per_block);
  // one row of 8 channels: (dy + addend) masked by y, accumulated; dyr stored
  auto row = [&](const long off, const uint4 vd, const uint4 vx, const uint4 vy, const uint4 va,
                 const uint32_t vm) {
    float fd[8], fx[8];
    unpack8(vd, fd);
    unpack8(vx, fx);
    if (addend) {
      float fa[8];
      unpack8(va, fa);
#pragma unroll
      for (int i = 0; i < 8; ++i) fd[i] += fa[i];
    }
    if (relu && ymask) {
#pragma unroll
      for (int i = 0; i < 8; ++i) fd[i] = (vm >> i) & 1u ? fd[i] : 0.f;
    } else if (relu) {
      float fy[8];
      unpack8(vy, fy);
#pragma unroll
      for (int i = 0; i < 8; ++i) fd[i] = fy[i] <= 0.f ? 0.f : fd[i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i] += fd[i];
      b[i] += fd[i] * (fx[i] - mu[i]) * rs[i];
    }
    if (dp_out) *(uint4*)(dp_out + off) = pack8(fd);
  };
  if (rl < rpb) {
    const uint4 z = make_uint4(0, 0, 0, 0);
    long r = r0 + rl;
    // 4 rows' loads in flight per thread before any use (the 2-tensor
    // non-residual case is otherwise latency-bound)
    constexpr int U = 4;
    for (; r + (U - 1) * rpb < r1; r += U * rpb) {
      uint4 vd[U], vx[U], vy[U], va[U];
      uint32_t vm[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long off = (r + u * rpb) * C + c0 + cg * 8;
        vd[u] = *(const uint4*)(dy + off);
        vx[u] = *(const uint4*)(x + off);
        vy[u] = relu && y ? *(const uint4*)(y + off) : z;
        va[u] = addend ? *(const uint4*)(addend + off) : z;
        vm[u] = relu && ymask ? ymask[off >> 3] : 0u;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) row((r + u * rpb) * C + c0 + cg * 8, vd[u], vx[u], vy[u], va[u], vm[u]);
    }
    for (; r < r1; r += rpb) {
      const long off = r * C + c0 + cg * 8;
      row(off, *(const uint4*)(dy + off), *(const uint4*)(x + off),
          relu && y ? *(const uint4*)(y + off) : z, addend ? *(const uint4*)(addend + off) : z,
          relu && ymask ? ymask[off >> 3] : 0u);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[threadIdx.x * 16 + i] = a[i]; red[threadIdx.x * 16 + 8 + i] = b[i]; }
  __syncthreads();
  if (rl == 0) {
    for (int j = 1; j < rpb; ++j) {
      const int t = j * tpr + cg;
#pragma unroll
      for (int i = 0; i < 8; ++i) { a[i] += red[t * 16 + i]; b[i] += red[t * 16 + 8 + i]; }
    }
  }
  bn_block_atomics(red, a, b, rl == 0, cg, cs, c0, C, sums);
}

// dx = g*rstd*(dyr - S/M - xhat*Q/M) = k1*dyr + k2*xhat + k3 with S, Q from
// the sums; blocks of row range 0 accumulate dgamma += Q, dbeta += S
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ addend, const bf16_t* __restrict__ y,
    const bf16_t* __restrict__ x, long M, int C, long rows_per_block, const double* __restrict__ sums,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ gamma,
    float* __restrict__ dgamma, float* __restrict__ dbeta, bf16_t* __restrict__ dx,
    bf16_t* __restrict__ dres, int relu, const uint8_t* __restrict__ ymask) {
  __shared__ float s_k[4][BN_SLAB];     // k1, k2, k3, mean
  const int c0 = blockIdx.y * BN_SLAB;
  const int cs = min(BN_SLAB, C - c0);
  const int t = threadIdx.x;
  if (t < cs) {
    const int c = c0 + t;
    double Sd, Qd;
    bn_shard_sum(sums, C, c, Sd, Qd);
    const float S = (float)Sd, Q = (float)Qd;
    const float rs = rstd[c], gr = gamma[c] * rs;
    // k2 multiplies (x - mean) directly: rstd folded in
    s_k[0][t] = gr;
    s_k[1][t] = -gr * Q / (float)M * rs;
    s_k[2][t] = -gr * S / (float)M;
    s_k[3][t] = mean[c];
    if (blockIdx.x == 0) {
      if (dgamma) dgamma[c] += Q;
      if (dbeta) dbeta[c] += S;
    }
  }
  __syncthreads();
  const int vs = cs / 8, rpp = 256 / vs;
  const int v = t % vs, rl = t / vs;
  if (rl >= rpp) return;
  float k1[8], k2[8], k3[8], mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k1[j] = s_k[0][v * 8 + j]; k2[j] = s_k[1][v * 8 + j]; k3[j] = s_k[2][v * 8 + j]; mu[j] = s_k[3][v * 8 + j];
  }
  auto one = [&](const long off, const uint4 vd, const uint4 vx, const uint4 vy, const uint4 va,
                 const uint32_t vm) {
    float fd[8], fx[8];
    unpack8(vd, fd);
    unpack8(vx, fx);
    if (addend) {
      float fa[8];
      unpack8(va, fa);
#pragma unroll
      for (int j = 0; j < 8; ++j) fd[j] += fa[j];
    }
    if (relu && ymask) {
#pragma unroll
      for (int j = 0; j < 8; ++j) fd[j] = (vm >> j) & 1u ? fd[j] : 0.f;
    } else if (relu) {
      float fy[8];
      unpack8(vy, fy);
#pragma unroll
      for (int j = 0; j < 8; ++j) fd[j] = fy[j] <= 0.f ? 0.f : fd[j];
    }
    if (dres) *(uint4*)(dres + off) = pack8(fd);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = k1[j] * fd[j] + k2[j] * (fx[j] - mu[j]) + k3[j];
    *(uint4*)(dx + off) = pack8(o);
  };
  const uint4 z = make_uint4(0, 0, 0, 0);
  const long r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  const long col = c0 + v * 8;
  long r = r0 + rl;
  for (; r + rpp < r1; r += 2 * rpp) {
    uint4 vd[2], vx[2], vy[2], va[2];
    uint32_t vm[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long off = (r + u * rpp) * C + col;
      vd[u] = *(const uint4*)(dy + off);
      vx[u] = *(const uint4*)(x + off);
      vy[u] = relu && y ? *(const uint4*)(y + off) : z;
      va[u] = addend ? *(const uint4*)(addend + off) : z;
      vm[u] = relu && ymask ? ymask[off >> 3] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) one((r + u * rpp) * C + col, vd[u], vx[u], vy[u], va[u], vm[u]);
  }
  if (r < r1) {
    const long off = r * C + col;
    one(off, *(const uint4*)(dy + off), *(const uint4*)(x + off), relu && y ? *(const uint4*)(y + off) : z,
        addend ? *(const uint4*)(addend + off) : z, relu && ymask ? ymask[off >> 3] : 0u);
  }
}

void bn_forward(const bf16_t* x, const bf16_t* res, bf16_t* y, long M, int C, float eps,
                float momentum, const float* gamma, const float* beta, float* run_mean,
                float* run_var, float* save_mean, float* save_rstd, int relu, double* sums,
                int sums_ready, uint8_t* ymask, hipStream_t s) {
  if (!sums_ready) {
    const BnRed g = bn_reduce_grid(M, C);
    hipLaunchKernelGGL(bn_stats_kernel, g.grid, dim3(256), 0, s, x, M, C, g.rows_per_block, g.sw, sums);
  }
  const BnGrid g = bn_apply_grid(M, C);
  hipLaunchKernelGGL(bn_apply_kernel, g.grid, dim3(256), 0, s, x, res, y, M, C, g.rows_per_block,
                     (const double*)sums, gamma, beta, eps, momentum, save_mean, save_rstd, run_mean,
                     run_var, relu, ymask);
}

// inference: scale / shift given (no statistics)
__global__ void __launch_bounds__(256) bn_infer_kernel(const bf16_t* __restrict__ x,
                                                        const bf16_t* __restrict__ res,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ shift,
                                                        bf16_t* __restrict__ y, long total8, int C,
                                                        int relu) {
  const int cg8 = C / 8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total8;
       i += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cg8) * 8;
    float f[8], rr[8];
    unpack8(((const uint4*)x)[i], f);
    if (res) unpack8(((const uint4*)res)[i], rr);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = f[j] * scale[c0 + j] + shift[c0 + j];
      if (res) v += rr[j];
      if (relu) v = fmaxf(v, 0.f);
      f[j] = v;
    }
    ((uint4*)y)[i] = pack8(f);
  }
}

void bn_infer(const bf16_t* x, const bf16_t* res, bf16_t* y, long M, int C, const float* scale,
              const float* shift, int relu, hipStream_t s) {
  const long total8 = M * C / 8;
  long b = (total8 + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(bn_infer_kernel, dim3((unsigned)b), dim3(256), 0, s, x, res, scale, shift, y,
                     total8, C, relu);
}

void bn_backward(const bf16_t* dy, const bf16_t* addend, const bf16_t* y, const bf16_t* x,
                 const float* mean, const float* rstd, const float* gamma, long M, int C, int relu,
                 bf16_t* dx, bf16_t* dres, float* dgamma, float* dbeta, double* sums,
                 int sums_ready, const uint8_t* ymask, hipStream_t s) {
  if (!sums_ready) {
    // residual BN: the reduce pass materialises dyr into dres; the apply pass
    // then runs on (dres, x) as a plain BN backward
    const BnRed g = bn_reduce_grid(M, C);
    hipLaunchKernelGGL(bn_bwd_reduce_kernel, g.grid, dim3(256), 0, s, dy, addend, y, x, mean, rstd, M,
                       C, g.rows_per_block, g.sw, relu, sums, dres, ymask);
    if (dres) {
      dy = dres;
      addend = nullptr;
      y = nullptr;
      ymask = nullptr;
      relu = 0;
      dres = nullptr;
    }
  }
  const BnGrid g = bn_apply_grid(M, C);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, g.grid, dim3(256), 0, s, dy, addend, y, x, M, C,
                     g.rows_per_block, (const double*)sums, mean, rstd, gamma, dgamma, dbeta, dx, dres,
                     relu, ymask);
}

// ---------------------------------------------------------------- LayerNorm
// One wave per row; D <= 64*8*ROWVEC. Vectorized 8 bf16 per lane-step.
template <int VEC>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const bf16_t* __restrict__ x,
                                                      const float* __restrict__ g,
                                                      const float* __restrict__ b,
                                                      bf16_t* __restrict__ y,
                                                      float* __restrict__ mean_o,
                                                      float* __restrict__ rstd_o, long rows, int D,
                                                      float eps, const bf16_t* __restrict__ addend,
                                                      bf16_t* __restrict__ sum_out) {
  const int lane = threadIdx.x & 63;
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16_t* xr = x + row * D;
  float f[VEC][8];
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    const int c = (v * 64 + lane) * 8;
    if (c < D) {
      unpack8(*(const uint4*)(xr + c), f[v]);
      if (addend) {
        // fused residual add: the bf16-rounded sum is both stored (the
        // residual stream) and normalised -- as an add pass + LN would see it
        float a[8];
        unpack8(*(const uint4*)(addend + row * D + c), a);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[v][j] += a[j];
        const uint4 pk = pack8(f[v]);
        *(uint4*)(sum_out + row * D + c) = pk;
        unpack8(pk, f[v]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) f[v][j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += f[v][j];
  }
  const float mu = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    const int c = (v * 64 + lane) * 8;
    if (c < D) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = f[v][j] - mu; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / D + eps);
  if (lane == 0) { mean_o[row] = mu; rstd_o[row] = rstd; }
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    const int c = (v * 64 + lane) * 8;
    if (c < D) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (f[v][j] - mu) * rstd * g[c + j] + b[c + j];
      *(uint4*)(y + row * D + c) = pack8(o);
    }
  }
}

template <int VEC>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const bf16_t* __restrict__ dy,
                                                      const bf16_t* __restrict__ x,
                                                      const float* __restrict__ g,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ rstd,
                                                      bf16_t* __restrict__ dx,
                                                      const bf16_t* __restrict__ addend,
                                                      float* __restrict__ part, long rows,
                                                      int D, int rows_per_block) {
  // each wave processes rows_per_block/4 rows, accumulating dgamma/dbeta in
  // registers; the 4 waves combine through LDS and the block writes ONE
  // partial row [2*D] (no atomics; a column-reduce kernel finishes).
  __shared__ float red[4 * 2 * VEC * 64 * 8];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  float dgacc[VEC][8], dbacc[VEC][8];
#pragma unroll
  for (int v = 0; v < VEC; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) dgacc[v][j] = dbacc[v][j] = 0.f;
  const long r0 = (long)blockIdx.x * rows_per_block;
  for (long row = r0 + w; row < min(rows, r0 + rows_per_block); row += 4) {
    const float mu = mean[row], rs = rstd[row];
    float fx[VEC][8], fd[VEC][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      const int c = (v * 64 + lane) * 8;
      if (c < D) {
        unpack8(*(const uint4*)(x + row * D + c), fx[v]);
        unpack8(*(const uint4*)(dy + row * D + c), fd[v]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (fx[v][j] - mu) * rs;
          fx[v][j] = xh;
          const float gd = fd[v][j] * g[c + j];
          s1 += gd;
          s2 += gd * xh;
          dgacc[v][j] += fd[v][j] * xh;
          dbacc[v][j] += fd[v][j];
        }
      }
    }
    s1 = wave_sum(s1) / D;
    s2 = wave_sum(s2) / D;
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      const int c = (v * 64 + lane) * 8;
      if (c < D) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (fd[v][j] * g[c + j] - s1 - fx[v][j] * s2);
        if (addend) {                      // + the residual branch's gradient (fused skip)
          float a[8];
          unpack8(*(const uint4*)(addend + row * D + c), a);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += a[j];
        }
        *(uint4*)(dx + row * D + c) = pack8(o);
      }
    }
  }
  // LDS layout: [wave][2][VEC*64*8]
  const int W = VEC * 64 * 8;
#pragma unroll
  for (int v = 0; v < VEC; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = (v * 64 + lane) * 8 + j;
      red[(w * 2 + 0) * W + c] = dgacc[v][j];
      red[(w * 2 + 1) * W + c] = dbacc[v][j];
    }
  __syncthreads();
  float* out = part + (long)blockIdx.x * 2 * D;
  for (int c = threadIdx.x; c < D; c += 256) {
    float g = 0.f, b = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) { g += red[(k * 2) * W + c]; b += red[(k * 2 + 1) * W + c]; }
    out[c] = g;
    out[D + c] = b;
  }
}


void ln_forward(const bf16_t* x, const float* g, const float* b, bf16_t* y, float* mean,
                float* rstd, long rows, int D, float eps, hipStream_t s, const bf16_t* addend,
                bf16_t* sum_out) {
  const int blocks = (int)((rows + 3) / 4);
  if (D <= 512) hipLaunchKernelGGL(ln_fwd_kernel<1>, dim3(blocks), dim3(256), 0, s, x, g, b, y, mean, rstd, rows, D, eps, addend, sum_out);
  else if (D <= 1024) hipLaunchKernelGGL(ln_fwd_kernel<2>, dim3(blocks), dim3(256), 0, s, x, g, b, y, mean, rstd, rows, D, eps, addend, sum_out);
  else hipLaunchKernelGGL(ln_fwd_kernel<4>, dim3(blocks), dim3(256), 0, s, x, g, b, y, mean, rstd, rows, D, eps, addend, sum_out);
}

int ln_backward_partial(const bf16_t* dy, const bf16_t* x, const float* g, const float* mean,
                        const float* rstd, bf16_t* dx, const bf16_t* addend, float* ws, long rows, int D,
                        hipStream_t s) {
  // ws: LN_MAX_BLOCKS * 2 * D floats of per-block partial dgamma / dbeta
  int rpb = (int)((rows + LN_MAX_BLOCKS - 1) / LN_MAX_BLOCKS);
  rpb = ((rpb + 3) / 4) * 4;
  if (rpb < 8) rpb = 8;
  const int blocks = (int)((rows + rpb - 1) / rpb);
  if (D <= 512) hipLaunchKernelGGL(ln_bwd_kernel<1>, dim3(blocks), dim3(256), 0, s, dy, x, g, mean, rstd, dx, addend, ws, rows, D, rpb);
  else if (D <= 1024) hipLaunchKernelGGL(ln_bwd_kernel<2>, dim3(blocks), dim3(256), 0, s, dy, x, g, mean, rstd, dx, addend, ws, rows, D, rpb);
  else hipLaunchKernelGGL(ln_bwd_kernel<4>, dim3(blocks), dim3(256), 0, s, dy, x, g, mean, rstd, dx, addend, ws, rows, D, rpb);
  return blocks;
}

void ln_backward(const bf16_t* dy, const bf16_t* x, const float* g, const float* mean,
                 const float* rstd, bf16_t* dx, const bf16_t* addend, float* dg, float* db,
                 float* ws, long rows, int D, hipStream_t s) {
  const int blocks = ln_backward_partial(dy, x, g, mean, rstd, dx, addend, ws, rows, D, s);
  col_reduce_acc(ws, blocks, 2 * D, dg, db, D, s);
}

}  // namespace tam
