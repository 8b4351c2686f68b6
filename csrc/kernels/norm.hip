// tiresias_amd — BatchNorm (NHWC, training) and LayerNorm kernels.
//
// BatchNorm is split into a stats pass (per-channel sum / sum-of-squares,
// fp32 per block -> fp64 global atomics so E[x^2]-E[x]^2 does not cancel at
// N*H*W ~ 10^5) and a fused apply pass (scale/shift + optional residual add +
// optional ReLU) reading 16 B per lane. Backward mirrors it: one reduction
// pass producing dgamma/dbeta (and the two row-means the input gradient
// needs), one fused pass producing dx (and the residual-branch gradient).
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

void col_reduce_f64(const float* part, int nblk, int W, double* out, hipStream_t s) {
  hipLaunchKernelGGL(col_reduce_kernel<0>, dim3((W + 15) / 16), dim3(256), 0, s, part, nblk, W, out,
                     (float*)nullptr, (float*)nullptr, W);
}
void col_reduce_acc(const float* part, int nblk, int W, float* out0, float* out1, int split,
                    hipStream_t s) {
  hipLaunchKernelGGL(col_reduce_kernel<1>, dim3((W + 15) / 16), dim3(256), 0, s, part, nblk, W,
                     (double*)nullptr, out0, out1, split);
}

// ---------------------------------------------------------------- BN stats
// grid.x blocks each own a contiguous row range; thread = (row lane, 8-ch group)
__global__ void __launch_bounds__(256) bn_stats_kernel(const bf16_t* __restrict__ x, long M, int C,
                                                        long rows_per_block,
                                                        float* __restrict__ part) {
  __shared__ float red[256 * 16];
  const int tpr = C / 8;                 // threads per row
  const int rpb = 256 / tpr;             // rows per pass (C <= 2048)
  const int cg = threadIdx.x % tpr, rl = threadIdx.x / tpr;
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
    // one partial row per block: no atomics, deterministic
    float* ps = part + (long)blockIdx.x * 2 * C + cg * 8;
    float* pq = ps + C;
#pragma unroll
    for (int i = 0; i < 8; ++i) { ps[i] = s[i]; pq[i] = q[i]; }
  }
}

// Column reduce of the [nblk][2C] partial rows (fp64) fused with the
// per-channel finalize: BWD=0 -> mean/rstd, scale/shift, running stats;
// BWD=1 -> dgamma/dbeta and the k1/k2/k3 coefficients of the apply pass.
// One launch instead of col_reduce + finalize (each ~5 us of a tiny grid).
// 1024 threads = 16 columns x 64 row lanes, 4 rows in flight per lane: the
// pass is latency-bound (one dependent kernel per BN), so more lanes per
// column, not more columns per block
template <int BWD>
__global__ void __launch_bounds__(1024) bn_reduce_finalize_kernel(
    const float* __restrict__ part, int nblk, long M, int C, float eps, float momentum,
    const float* __restrict__ gamma, const float* __restrict__ beta_or_rstd,
    float* __restrict__ o0, float* __restrict__ o1, float* __restrict__ o2,
    float* __restrict__ o3, float* __restrict__ o4, float* __restrict__ o5) {
  constexpr int RL = 64;
  __shared__ double red[2][RL][17];
  const int cx = threadIdx.x & 15, ly = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cx;
  const int W = 2 * C;
  double s = 0.0, q = 0.0;
  if (c < C) {
    int b = ly;
    for (; b + 3 * RL < nblk; b += 4 * RL) {
      float v[4], w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = part[(long)(b + u * RL) * W + c];
        w[u] = part[(long)(b + u * RL) * W + C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { s += (double)v[u]; q += (double)w[u]; }
    }
    for (; b < nblk; b += RL) {
      s += (double)part[(long)b * W + c];
      q += (double)part[(long)b * W + C + c];
    }
  }
  red[0][ly][cx] = s;
  red[1][ly][cx] = q;
  __syncthreads();
  if (ly != 0 || c >= C) return;
  double S = 0.0, Q = 0.0;
#pragma unroll 8
  for (int k = 0; k < RL; ++k) { S += red[0][k][cx]; Q += red[1][k][cx]; }
  if (BWD == 0) {
    // o0 mean, o1 rstd, o2 scale, o3 shift, o4 run_mean, o5 run_var
    const double mean = S / (double)M;
    double var = Q / (double)M - mean * mean;
    if (var < 0) var = 0;
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    o0[c] = (float)mean;
    o1[c] = rstd;
    const float sc = gamma[c] * rstd;
    o2[c] = sc;
    o3[c] = beta_or_rstd[c] - (float)mean * sc;
    if (o4) {
      const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
      o4[c] = (1.f - momentum) * o4[c] + momentum * (float)mean;
      o5[c] = (1.f - momentum) * o5[c] + momentum * (float)unb;
    }
  } else {
    // o0 dgamma, o1 dbeta (accumulate), o2 k1, o3 k2, o4 k3
    const float a = (float)S, bb = (float)Q;
    if (o0) o0[c] += bb;
    if (o1) o1[c] += a;
    const float gr = gamma[c] * beta_or_rstd[c];
    o2[c] = gr;
    o3[c] = -gr * bb / (float)M;
    o4[c] = -gr * a / (float)M;
  }
}

// mean/rstd + fused scale/shift + running-stat update
__global__ void bn_finalize_kernel(const double* __restrict__ sums, long M, int C, float eps,
                                   float momentum,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                   float* __restrict__ scale, float* __restrict__ shift,
                                   float* __restrict__ run_mean, float* __restrict__ run_var) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double mean = sums[c] / (double)M;
  double var = sums[C + c] / (double)M - mean * mean;
  if (var < 0) var = 0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  mean_out[c] = (float)mean;
  rstd_out[c] = rstd;
  const float sc = gamma[c] * rstd;
  scale[c] = sc;
  shift[c] = beta[c] - (float)mean * sc;
  if (run_mean) {
    const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unb;
  }
}

// y = x*scale + shift (+res) (relu), 8 channels per thread
__global__ void __launch_bounds__(256) bn_apply_kernel(const bf16_t* __restrict__ x,
                                                        const bf16_t* __restrict__ res,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ shift,
                                                        bf16_t* __restrict__ y, long total8, int C,
                                                        int relu) {
  const int cg8 = C / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  auto one = [&](const long ii, const uint4 vx, const uint4 vr) {
    const int c0 = (int)(ii % cg8) * 8;
    float f[8], rr[8];
    unpack8(vx, f);
    if (res) unpack8(vr, rr);
    const float4 sa = *(const float4*)(scale + c0), sb = *(const float4*)(scale + c0 + 4);
    const float4 ha = *(const float4*)(shift + c0), hb = *(const float4*)(shift + c0 + 4);
    const float sc[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
    const float sh[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = f[j] * sc[j] + sh[j];
      if (res) v += rr[j];
      if (relu) v = fmaxf(v, 0.f);
      f[j] = v;
    }
    ((uint4*)y)[ii] = pack8(f);
  };
  const uint4 z = make_uint4(0, 0, 0, 0);
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  // 2 vectors' loads in flight per thread before any use
  constexpr int U = 2;
  for (; i + (U - 1) * stride < total8; i += U * stride) {
    uint4 vx[U], vr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      vx[u] = ((const uint4*)x)[i + u * stride];
      vr[u] = res ? ((const uint4*)res)[i + u * stride] : z;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(i + u * stride, vx[u], vr[u]);
  }
  for (; i < total8; i += stride) one(i, ((const uint4*)x)[i], res ? ((const uint4*)res)[i] : z);
}

// ---------------------------------------------------------------- BN backward
// dyr = (dy + addend) * (y > 0 if relu); accum sum(dyr), sum(dyr * xhat) per
// channel. dp_out (residual BNs): dyr is also stored -- it IS the residual
// branch's gradient, and the apply pass then reads dyr + x only (no dy,
// addend, y re-reads, no second dres write: 2 passes of the tensor saved)
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ addend, const bf16_t* __restrict__ y,
    const bf16_t* __restrict__ x, const float* __restrict__ mean, const float* __restrict__ rstd, long M,
    int C, long rows_per_block, int relu, float* __restrict__ part, bf16_t* __restrict__ dp_out) {
  __shared__ float red[256 * 16];
  const int tpr = C / 8, rpb = 256 / tpr;
  const int cg = threadIdx.x % tpr, rl = threadIdx.x / tpr;
  float a[8], b[8], mu[8], rs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { a[i] = b[i] = 0.f; mu[i] = mean[cg * 8 + i]; rs[i] = rstd[cg * 8 + i]; }
  const long r0 = blockIdx.x * rows_per_block;
  const long r1 = min(M, r0 + rows_per_block);
  // one row of 8 channels: (dy + addend) masked by y, accumulated; dyr stored
  auto row = [&](const long off, const uint4 vd, const uint4 vx, const uint4 vy, const uint4 va) {
    float fd[8], fx[8];
    unpack8(vd, fd);
    unpack8(vx, fx);
    if (addend) {
      float fa[8];
      unpack8(va, fa);
#pragma unroll
      for (int i = 0; i < 8; ++i) fd[i] += fa[i];
    }
    if (relu) {
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
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long off = (r + u * rpb) * C + cg * 8;
        vd[u] = *(const uint4*)(dy + off);
        vx[u] = *(const uint4*)(x + off);
        vy[u] = relu ? *(const uint4*)(y + off) : z;
        va[u] = addend ? *(const uint4*)(addend + off) : z;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) row((r + u * rpb) * C + cg * 8, vd[u], vx[u], vy[u], va[u]);
    }
    for (; r < r1; r += rpb) {
      const long off = r * C + cg * 8;
      row(off, *(const uint4*)(dy + off), *(const uint4*)(x + off),
          relu ? *(const uint4*)(y + off) : z, addend ? *(const uint4*)(addend + off) : z);
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
    float* pa = part + (long)blockIdx.x * 2 * C + cg * 8;
    float* pb = pa + C;
#pragma unroll
    for (int i = 0; i < 8; ++i) { pa[i] = a[i]; pb[i] = b[i]; }
  }
}

// dgamma/dbeta accumulate into fp32 grads; coefficient prep for the apply pass
__global__ void bn_bwd_finalize_kernel(const double* __restrict__ sums, long M, int C,
                                       const float* __restrict__ gamma,
                                       const float* __restrict__ rstd, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta, float* __restrict__ k1,
                                       float* __restrict__ k2, float* __restrict__ k3) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float a = (float)sums[c], b = (float)sums[C + c];
  if (dgamma) dgamma[c] += b;
  if (dbeta) dbeta[c] += a;
  // dx = g*rstd*(dyr - a/M - xhat*b/M) = k1*dyr + k2*xhat + k3
  const float gr = gamma[c] * rstd[c];
  k1[c] = gr;
  k2[c] = -gr * b / (float)M;
  k3[c] = -gr * a / (float)M;
}

__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ addend, const bf16_t* __restrict__ y,
    const bf16_t* __restrict__ x,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ k1,
    const float* __restrict__ k2, const float* __restrict__ k3, bf16_t* __restrict__ dx,
    bf16_t* __restrict__ dres, long total8, int C, int relu) {
  const int cg8 = C / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  auto one = [&](const long ii, const uint4 vd, const uint4 vx, const uint4 vy, const uint4 va) {
    const int c0 = (int)(ii % cg8) * 8;
    float fd[8], fx[8];
    unpack8(vd, fd);
    unpack8(vx, fx);
    if (addend) {
      float fa[8];
      unpack8(va, fa);
#pragma unroll
      for (int j = 0; j < 8; ++j) fd[j] += fa[j];
    }
    if (relu) {
      float fy[8];
      unpack8(vy, fy);
#pragma unroll
      for (int j = 0; j < 8; ++j) fd[j] = fy[j] <= 0.f ? 0.f : fd[j];
    }
    if (dres) ((uint4*)dres)[ii] = pack8(fd);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      const float xh = (fx[j] - mean[c]) * rstd[c];
      o[j] = k1[c] * fd[j] + k2[c] * xh + k3[c];
    }
    ((uint4*)dx)[ii] = pack8(o);
  };
  const uint4 z = make_uint4(0, 0, 0, 0);
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  // 2 vectors' loads in flight per thread before any use
  constexpr int U = 2;
  for (; i + (U - 1) * stride < total8; i += U * stride) {
    uint4 vd[U], vx[U], vy[U], va[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long ii = i + u * stride;
      vd[u] = ((const uint4*)dy)[ii];
      vx[u] = ((const uint4*)x)[ii];
      vy[u] = relu ? ((const uint4*)y)[ii] : z;
      va[u] = addend ? ((const uint4*)addend)[ii] : z;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(i + u * stride, vd[u], vx[u], vy[u], va[u]);
  }
  for (; i < total8; i += stride)
    one(i, ((const uint4*)dy)[i], ((const uint4*)x)[i], relu ? ((const uint4*)y)[i] : z,
        addend ? ((const uint4*)addend)[i] : z);
}

// elementwise grids: one thread per 16-B vector up to 2048 blocks (8 per CU);
// measured: fewer, 4x-unrolled blocks (n / 1024) were slower on ResNet-50
static int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

static long bn_rows_per_block(long M, int C) {
  // <= BN_MAX_BLOCKS partial rows (2 blocks per CU on 256 CUs); each block
  // streams >= 4 passes of its thread grid so the loads stay 16 B/lane
  long rpb = (M + BN_MAX_BLOCKS - 1) / BN_MAX_BLOCKS;
  const long minr = 256 / (C / 8) * 4;
  if (rpb < minr) rpb = minr;
  return rpb;
}

void bn_forward(const bf16_t* x, const bf16_t* res, bf16_t* y, long M, int C, float eps,
                float momentum, const float* gamma, const float* beta, float* run_mean,
                float* run_var, float* save_mean, float* save_rstd, float* ws_f, int relu,
                const float* part_in, int nblk_in, hipStream_t s) {
  // ws_f: 2*C floats scale/shift | 2*C doubles column sums | BN_MAX_BLOCKS*2*C partials
  // part_in: [nblk_in][2C] partial rows already produced (conv epilogue): no stats pass
  const long rpb = bn_rows_per_block(M, C);
  int nb = (int)((M + rpb - 1) / rpb);
  double* sums = (double*)(ws_f + 2 * C);
  const float* part = ws_f + 6 * C;
  (void)sums;
  if (part_in && nblk_in > 0) {
    part = part_in;
    nb = nblk_in;
  } else {
    hipLaunchKernelGGL(bn_stats_kernel, dim3(nb), dim3(256), 0, s, x, M, C, rpb, ws_f + 6 * C);
  }
  hipLaunchKernelGGL(bn_reduce_finalize_kernel<0>, dim3((C + 15) / 16), dim3(1024), 0, s, part, nb, M,
                     C, eps, momentum, gamma, beta, save_mean, save_rstd, ws_f, ws_f + C, run_mean,
                     run_var);
  const long total8 = M * C / 8;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for(total8)), dim3(256), 0, s, x, res, ws_f,
                     ws_f + C, y, total8, C, relu);
}

void bn_infer(const bf16_t* x, const bf16_t* res, bf16_t* y, long M, int C, const float* scale,
              const float* shift, int relu, hipStream_t s) {
  const long total8 = M * C / 8;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for(total8)), dim3(256), 0, s, x, res, scale,
                     shift, y, total8, C, relu);
}

void bn_backward(const bf16_t* dy, const bf16_t* addend, const bf16_t* y, const bf16_t* x,
                 const float* mean, const float* rstd, const float* gamma, long M, int C, int relu,
                 bf16_t* dx, bf16_t* dres, float* dgamma, float* dbeta, float* ws_f, hipStream_t s) {
  // ws_f: 4*C floats k1/k2/k3(+pad) | 2*C doubles column sums | BN_MAX_BLOCKS*2*C partials
  const long rpb = bn_rows_per_block(M, C);
  const int nb = (int)((M + rpb - 1) / rpb);
  double* sums = (double*)(ws_f + 4 * C);
  float* part = ws_f + 8 * C;
  // residual BN: the reduce pass materialises dyr into dres; the apply pass
  // then runs on (dres, x) as a plain BN backward
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(nb), dim3(256), 0, s, dy, addend, y, x, mean, rstd, M,
                     C, rpb, relu, part, dres);
  if (dres) {
    dy = dres;
    addend = nullptr;
    y = nullptr;
    relu = 0;
    dres = nullptr;
  }
  (void)sums;
  hipLaunchKernelGGL(bn_reduce_finalize_kernel<1>, dim3((C + 15) / 16), dim3(1024), 0, s, part, nb, M,
                     C, 0.f, 0.f, gamma, rstd, dgamma, dbeta, ws_f, ws_f + C, ws_f + 2 * C,
                     (float*)nullptr);
  const long total8 = M * C / 8;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(total8)), dim3(256), 0, s, dy, addend, y, x,
                     mean, rstd, ws_f, ws_f + C, ws_f + 2 * C, dx, dres, total8, C, relu);
}

// BN backward whose reduction already happened in the consumer conv's dgrad
// epilogue (Epi::bnx): part = [nblk][2C] partial rows of sum(d) | sum(d*xhat)
// over the ReLU-masked output gradient d; finalize + one apply pass
void bn_backward_part(const bf16_t* dy, const bf16_t* x, const float* mean, const float* rstd,
                      const float* gamma, long M, int C, bf16_t* dx, float* dgamma, float* dbeta,
                      const float* part, int nblk, float* ws_f, hipStream_t s) {
  hipLaunchKernelGGL(bn_reduce_finalize_kernel<1>, dim3((C + 15) / 16), dim3(1024), 0, s, part, nblk, M,
                     C, 0.f, 0.f, gamma, rstd, dgamma, dbeta, ws_f, ws_f + C, ws_f + 2 * C,
                     (float*)nullptr);
  const long total8 = M * C / 8;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(total8)), dim3(256), 0, s, dy,
                     (const bf16_t*)nullptr, (const bf16_t*)nullptr, x, mean, rstd, ws_f, ws_f + C,
                     ws_f + 2 * C, dx, (bf16_t*)nullptr, total8, C, 0);
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
                                                      float eps) {
  const int lane = threadIdx.x & 63;
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16_t* xr = x + row * D;
  float f[VEC][8];
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    const int c = (v * 64 + lane) * 8;
    if (c < D) unpack8(*(const uint4*)(xr + c), f[v]);
    else {
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
                float* rstd, long rows, int D, float eps, hipStream_t s) {
  const int blocks = (int)((rows + 3) / 4);
  if (D <= 512) hipLaunchKernelGGL(ln_fwd_kernel<1>, dim3(blocks), dim3(256), 0, s, x, g, b, y, mean, rstd, rows, D, eps);
  else if (D <= 1024) hipLaunchKernelGGL(ln_fwd_kernel<2>, dim3(blocks), dim3(256), 0, s, x, g, b, y, mean, rstd, rows, D, eps);
  else hipLaunchKernelGGL(ln_fwd_kernel<4>, dim3(blocks), dim3(256), 0, s, x, g, b, y, mean, rstd, rows, D, eps);
}

void ln_backward(const bf16_t* dy, const bf16_t* x, const float* g, const float* mean,
                 const float* rstd, bf16_t* dx, const bf16_t* addend, float* dg, float* db,
                 float* ws, long rows, int D, hipStream_t s) {
  // ws: LN_MAX_BLOCKS * 2 * D floats of per-block partial dgamma / dbeta
  int rpb = (int)((rows + LN_MAX_BLOCKS - 1) / LN_MAX_BLOCKS);
  rpb = ((rpb + 3) / 4) * 4;
  if (rpb < 8) rpb = 8;
  const int blocks = (int)((rows + rpb - 1) / rpb);
  if (D <= 512) hipLaunchKernelGGL(ln_bwd_kernel<1>, dim3(blocks), dim3(256), 0, s, dy, x, g, mean, rstd, dx, addend, ws, rows, D, rpb);
  else if (D <= 1024) hipLaunchKernelGGL(ln_bwd_kernel<2>, dim3(blocks), dim3(256), 0, s, dy, x, g, mean, rstd, dx, addend, ws, rows, D, rpb);
  else hipLaunchKernelGGL(ln_bwd_kernel<4>, dim3(blocks), dim3(256), 0, s, dy, x, g, mean, rstd, dx, addend, ws, rows, D, rpb);
  col_reduce_acc(ws, blocks, 2 * D, dg, db, D, s);
}

}  // namespace tam
