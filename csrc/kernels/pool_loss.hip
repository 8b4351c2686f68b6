// tiresias_amd — pooling (NHWC), fused softmax cross-entropy, embedding and
// small elementwise kernels.
#include "tam/common.h"
#include "tam/kernels.h"

namespace tam {

static int grid_cap(long n, int cap = 4096) {
  long b = (n + 255) / 256;
  if (b > cap) b = cap;
  return (int)(b < 1 ? 1 : b);
}

// ------------------------------------------------------------------ max pool
// y[n,p,q,c] = max over window; idx stores the argmax tap (r*S+s) as uint8.
__global__ void maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                   uint8_t* __restrict__ idx, int N, int H, int W, int C, int P,
                                   int Q, int R, int S, int st, int pad) {
  const long total = (long)N * P * Q * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
    const int q = (int)(t % Q); t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float best = -INFINITY;
    int bi = 0;
    for (int r = 0; r < R; ++r) {
      const int h = p * st - pad + r;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int s = 0; s < S; ++s) {
        const int w = q * st - pad + s;
        if ((unsigned)w >= (unsigned)W) continue;
        const float v = bf2f(x[(((long)n * H + h) * W + w) * C + c]);
        if (v > best) { best = v; bi = r * S + s; }
      }
    }
    y[i] = f2bf(best);
    idx[i] = (uint8_t)bi;
  }
}

// gather-form backward: each input element sums the outputs whose argmax it is
__global__ void maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                   bf16_t* __restrict__ dx, int N, int H, int W, int C, int P,
                                   int Q, int R, int S, int st, int pad) {
  const long total = (long)N * H * W * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
    const int w = (int)(t % W); t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float acc = 0.f;
    for (int r = 0; r < R; ++r) {
      const int pn = h + pad - r;
      if (pn < 0 || pn % st) continue;
      const int p = pn / st;
      if (p >= P) continue;
      for (int s = 0; s < S; ++s) {
        const int qn = w + pad - s;
        if (qn < 0 || qn % st) continue;
        const int q = qn / st;
        if (q >= Q) continue;
        const long o = (((long)n * P + p) * Q + q) * C + c;
        if (idx[o] == r * S + s) acc += bf2f(dy[o]);
      }
    }
    dx[i] = f2bf(acc);
  }
}

// 8-channel vector forms (C % 8 == 0): one (n,h,w,8c) tuple per thread, 16 B
// loads of x/dy and 8 B loads of idx; index math amortised over 8 channels.
__global__ void maxpool_fwd8_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                    uint8_t* __restrict__ idx, int N, int H, int W, int C, int P,
                                    int Q, int R, int S, int st, int pad) {
  const int C8 = C / 8;
  const long total = (long)N * P * Q * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C8) * 8;
    long t = i / C8;
    const int q = (int)(t % Q); t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float best[8];
    uint32_t bi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; bi[k] = 0; }
    for (int r = 0; r < R; ++r) {
      const int h = p * st - pad + r;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int s = 0; s < S; ++s) {
        const int w = q * st - pad + s;
        if ((unsigned)w >= (unsigned)W) continue;
        const uint4 v = *(const uint4*)(x + (((long)n * H + h) * W + w) * C + c);
        const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float a = __uint_as_float(wv[k] << 16), b = __uint_as_float(wv[k] & 0xffff0000u);
          if (a > best[2 * k]) { best[2 * k] = a; bi[2 * k] = r * S + s; }
          if (b > best[2 * k + 1]) { best[2 * k + 1] = b; bi[2 * k + 1] = r * S + s; }
        }
      }
    }
    const long o = i * 8;
    *(uint4*)(y + o) = make_uint4(pack_bf2(best[0], best[1]), pack_bf2(best[2], best[3]),
                                  pack_bf2(best[4], best[5]), pack_bf2(best[6], best[7]));
    *(uint2*)(idx + o) = make_uint2(bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24),
                                    bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24));
  }
}

__global__ void maxpool_bwd8_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                    bf16_t* __restrict__ dx, int N, int H, int W, int C, int P,
                                    int Q, int R, int S, int st, int pad) {
  const int C8 = C / 8;
  const long total = (long)N * H * W * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C8) * 8;
    long t = i / C8;
    const int w = (int)(t % W); t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < R; ++r) {
      const int pn = h + pad - r;
      if (pn < 0 || pn % st) continue;
      const int p = pn / st;
      if (p >= P) continue;
      for (int s = 0; s < S; ++s) {
        const int qn = w + pad - s;
        if (qn < 0 || qn % st) continue;
        const int q = qn / st;
        if (q >= Q) continue;
        const long o = (((long)n * P + p) * Q + q) * C + c;
        const uint2 ix = *(const uint2*)(idx + o);
        const uint4 d = *(const uint4*)(dy + o);
        const uint32_t wd[4] = {d.x, d.y, d.z, d.w};
        const uint32_t tap = (uint32_t)(r * S + s);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t b = ((k < 4 ? ix.x : ix.y) >> (8 * (k & 3))) & 0xffu;
          const uint32_t wk = wd[k >> 1];
          const float g = __uint_as_float((k & 1) ? (wk & 0xffff0000u) : (wk << 16));
          if (b == tap) acc[k] += g;
        }
      }
    }
    *(uint4*)(dx + i * 8) = make_uint4(pack_bf2(acc[0], acc[1]), pack_bf2(acc[2], acc[3]),
                                       pack_bf2(acc[4], acc[5]), pack_bf2(acc[6], acc[7]));
  }
}

// 3x3 / stride 2 / pad 1 (the ResNet stem pool): an input pixel lies in 1, 2
// or 4 windows, found from the parities of h and w with no tap loop and no
// runtime division (the generic kernel above spends its time in the 9-tap
// loop's integer div / mod: 83 us for the 112x112x64 batch-64 stem, ~3x
// its bytes at HBM rate)
__global__ void __launch_bounds__(256) maxpool_bwd8_k3s2_kernel(const bf16_t* __restrict__ dy,
                                                                 const uint8_t* __restrict__ idx,
                                                                 bf16_t* __restrict__ dx, int N, int H, int W,
                                                                 int C8, int P, int Q) {
  const long total = (long)N * H * W * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C8) * 8;
    const long t = i / C8;
    const int w = (int)(t % W);
    const long t2 = t / W;
    const int h = (int)(t2 % H);
    const int n = (int)(t2 / H);
    // windows p with h = 2p - 1 + r, r in [0, 3): odd h -> p = (h+1)/2 (r=0)
    // and (h-1)/2 (r=2); even h -> p = h/2 (r=1)
    int ps[2], rs[2], np = 0;
    if (h & 1) {
      if ((h + 1) / 2 < P) { ps[np] = (h + 1) / 2; rs[np] = 0; ++np; }
      ps[np] = (h - 1) / 2; rs[np] = 2; ++np;
    } else {
      if (h / 2 < P) { ps[np] = h / 2; rs[np] = 1; ++np; }
    }
    int qs[2], ss[2], nq = 0;
    if (w & 1) {
      if ((w + 1) / 2 < Q) { qs[nq] = (w + 1) / 2; ss[nq] = 0; ++nq; }
      qs[nq] = (w - 1) / 2; ss[nq] = 2; ++nq;
    } else {
      if (w / 2 < Q) { qs[nq] = w / 2; ss[nq] = 1; ++nq; }
    }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int a = 0; a < np; ++a)
      for (int b = 0; b < nq; ++b) {
        const long o = (((long)n * P + ps[a]) * Q + qs[b]) * (C8 * 8) + c;
        const uint2 ix = *(const uint2*)(idx + o);
        const uint4 d = *(const uint4*)(dy + o);
        const uint32_t wd[4] = {d.x, d.y, d.z, d.w};
        const uint32_t tap = (uint32_t)(rs[a] * 3 + ss[b]);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t bb = ((k < 4 ? ix.x : ix.y) >> (8 * (k & 3))) & 0xffu;
          const uint32_t wk = wd[k >> 1];
          const float g = __uint_as_float((k & 1) ? (wk & 0xffff0000u) : (wk << 16));
          if (bb == tap) acc[k] += g;
        }
      }
    *(uint4*)(dx + i * 8) = make_uint4(pack_bf2(acc[0], acc[1]), pack_bf2(acc[2], acc[3]),
                                       pack_bf2(acc[4], acc[5]), pack_bf2(acc[6], acc[7]));
  }
}

// Non-overlapping windows (window == stride, no padding, the input an exact
// multiple of the window, C / 8 a power of two: VGG-16's 2x2 / s2 pools).
// One thread per (output pixel, 8 channels); the grid's y is the output row
// (n, p) and x walks that row's Q * C/8 tuples, so the index math is a mask
// and a shift -- the generic 8-channel kernels above spend most of their time
// in 64-bit runtime div / mod (VALU-bound: 0.91 VALU utilisation, PMC).
// Forward: same (dr, ds) scan order and strict '>' as the generic kernel, so
// ties pick the same tap. Backward: every input pixel lies in exactly one
// window, so it is written once (no accumulation, no tap loop).
__global__ void __launch_bounds__(256) maxpool_fwd_ws_kernel(const bf16_t* __restrict__ x,
                                                             bf16_t* __restrict__ y,
                                                             uint8_t* __restrict__ idx, int Q, int C,
                                                             int lc8, int st) {
  const int row = blockIdx.y;                     // n * P + p
  const int n_el = Q << lc8, m8 = (1 << lc8) - 1;
  const long W = (long)Q * st;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n_el; e += gridDim.x * blockDim.x) {
    const int c = (e & m8) * 8, q = e >> lc8;
    float best[8];
    uint32_t bi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; bi[k] = 0; }
    for (int r = 0; r < st; ++r) {
      const bf16_t* xr = x + (((long)row * st + r) * W + (long)q * st) * C + c;
      for (int s = 0; s < st; ++s) {
        const uint4 v = *(const uint4*)(xr + (long)s * C);
        const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
        const uint32_t tap = (uint32_t)(r * st + s);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float a = __uint_as_float(wv[k] << 16), b = __uint_as_float(wv[k] & 0xffff0000u);
          if (a > best[2 * k]) { best[2 * k] = a; bi[2 * k] = tap; }
          if (b > best[2 * k + 1]) { best[2 * k + 1] = b; bi[2 * k + 1] = tap; }
        }
      }
    }
    const long o = ((long)row * Q + q) * C + c;
    *(uint4*)(y + o) = make_uint4(pack_bf2(best[0], best[1]), pack_bf2(best[2], best[3]),
                                  pack_bf2(best[4], best[5]), pack_bf2(best[6], best[7]));
    *(uint2*)(idx + o) = make_uint2(bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24),
                                    bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24));
  }
}

__global__ void __launch_bounds__(256) maxpool_bwd_ws_kernel(const bf16_t* __restrict__ dy,
                                                             const uint8_t* __restrict__ idx,
                                                             bf16_t* __restrict__ dx, int Q, int C,
                                                             int lc8, int st) {
  const int row = blockIdx.y;
  const int n_el = Q << lc8, m8 = (1 << lc8) - 1;
  const long W = (long)Q * st;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n_el; e += gridDim.x * blockDim.x) {
    const int c = (e & m8) * 8, q = e >> lc8;
    const long o = ((long)row * Q + q) * C + c;
    const uint2 ix = *(const uint2*)(idx + o);
    const uint4 d = *(const uint4*)(dy + o);
    const uint32_t wd[4] = {d.x, d.y, d.z, d.w};
    for (int r = 0; r < st; ++r) {
      bf16_t* xr = dx + (((long)row * st + r) * W + (long)q * st) * C + c;
      for (int s = 0; s < st; ++s) {
        const uint32_t tap = (uint32_t)(r * st + s);
        uint32_t out[4];
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) {
          // the two bf16 of word k2 pass through where their window max was this tap
          const uint32_t b0 = ((k2 < 2 ? ix.x : ix.y) >> (16 * (k2 & 1))) & 0xffu;
          const uint32_t b1 = ((k2 < 2 ? ix.x : ix.y) >> (16 * (k2 & 1) + 8)) & 0xffu;
          out[k2] = (b0 == tap ? (wd[k2] & 0x0000ffffu) : 0u) | (b1 == tap ? (wd[k2] & 0xffff0000u) : 0u);
        }
        *(uint4*)(xr + (long)s * C) = make_uint4(out[0], out[1], out[2], out[3]);
      }
    }
  }
}

static int ilog2_exact(int v) {   // log2 of a power of two, else -1
  if (v <= 0 || (v & (v - 1))) return -1;
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

static bool pool_ws_ok(int H, int W, int C, int P, int Q, int R, int S, int st, int pad) {
  return C % 8 == 0 && ilog2_exact(C / 8) >= 0 && R == st && S == st && pad == 0 && st >= 1 && st <= 4 &&
         H == P * st && W == Q * st && P <= 65535;
}

static dim3 pool_ws_grid(int N, int P, int Q, int C) {
  const int per_row = Q * (C / 8);
  int bx = (per_row + 255) / 256;
  if (bx > 64) bx = 64;
  return dim3((unsigned)bx, (unsigned)(N * P));
}

// policy: 1 (default) the specialised kernels where they apply (3x3/s2/p1
// backward, window == stride), 0 the generic ones (A/B, tests)
static int g_pool_k3s2 = 1;
TAM_KNOB(g_pool_k3s2)
void maxpool_k3s2_policy(int p) { g_pool_k3s2 = p; }

void maxpool_forward(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int P,
                     int Q, int R, int S, int st, int pad, hipStream_t s) {
  if (g_pool_k3s2 && pool_ws_ok(H, W, C, P, Q, R, S, st, pad) && (long)N * P <= 65535) {
    hipLaunchKernelGGL(maxpool_fwd_ws_kernel, pool_ws_grid(N, P, Q, C), dim3(256), 0, s, x, y, idx, Q, C,
                       ilog2_exact(C / 8), st);
    return;
  }
  if (C % 8 == 0) {
    hipLaunchKernelGGL(maxpool_fwd8_kernel, dim3(grid_cap((long)N * P * Q * (C / 8))), dim3(256), 0,
                       s, x, y, idx, N, H, W, C, P, Q, R, S, st, pad);
    return;
  }
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_cap((long)N * P * Q * C)), dim3(256), 0, s, x, y,
                     idx, N, H, W, C, P, Q, R, S, st, pad);
}
void maxpool_backward(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C,
                      int P, int Q, int R, int S, int st, int pad, hipStream_t s) {
  if (C % 8 == 0 && g_pool_k3s2 && R == 3 && S == 3 && st == 2 && pad == 1 && P == (H - 1) / 2 + 1 &&
      Q == (W - 1) / 2 + 1) {
    hipLaunchKernelGGL(maxpool_bwd8_k3s2_kernel, dim3(grid_cap((long)N * H * W * (C / 8))), dim3(256), 0, s, dy,
                       idx, dx, N, H, W, C / 8, P, Q);
    return;
  }
  if (g_pool_k3s2 && pool_ws_ok(H, W, C, P, Q, R, S, st, pad) && (long)N * P <= 65535) {
    hipLaunchKernelGGL(maxpool_bwd_ws_kernel, pool_ws_grid(N, P, Q, C), dim3(256), 0, s, dy, idx, dx, Q, C,
                       ilog2_exact(C / 8), st);
    return;
  }
  if (C % 8 == 0) {
    hipLaunchKernelGGL(maxpool_bwd8_kernel, dim3(grid_cap((long)N * H * W * (C / 8))), dim3(256), 0,
                       s, dy, idx, dx, N, H, W, C, P, Q, R, S, st, pad);
    return;
  }
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_cap((long)N * H * W * C)), dim3(256), 0, s, dy,
                     idx, dx, N, H, W, C, P, Q, R, S, st, pad);
}

// ------------------------------------------------------------ global avgpool
// x [N][HW][C] -> y [N][C]; one thread per (n, c)
__global__ void avgpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int N,
                                   int HW, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i % C;
  float s = 0.f;
  for (int p = 0; p < HW; ++p) s += bf2f(x[((long)n * HW + p) * C + c]);
  y[i] = f2bf(s / HW);
}
__global__ void avgpool_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, int N,
                                   int HW, int C) {
  const long total = (long)N * HW * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int n = (int)(i / ((long)HW * C));
    dx[i] = f2bf(bf2f(dy[(long)n * C + c]) / HW);
  }
}
void avgpool_forward(const bf16_t* x, bf16_t* y, int N, int HW, int C, hipStream_t s) {
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((N * C + 255) / 256), dim3(256), 0, s, x, y, N, HW, C);
}
void avgpool_backward(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t s) {
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_cap((long)N * HW * C)), dim3(256), 0, s, dy, dx,
                     N, HW, C);
}

// ------------------------------------------------- softmax cross-entropy fused
// One 256-thread block per row. Forward and backward in one kernel: the loss
// is the graph's sink, so dlogits = (softmax - target) * grad_scale is known.
// Label smoothing eps: target = (1-eps) onehot + eps/V. ignore_index rows
// contribute 0 loss / 0 grad.
// tm_b > 0: the logits rows are time-major (row r = s * tm_b + b) while the
// labels stay [tm_b][S] batch-major: row r reads labels[b * S + s] (no
// transposed copy of the labels, S = rows / tm_b)
__device__ __forceinline__ long tm_index(long r, long rows, long tm_b) {
  return tm_b > 0 ? (r % tm_b) * (rows / tm_b) + r / tm_b : r;
}

__global__ void __launch_bounds__(256) xent_kernel(const bf16_t* __restrict__ logits,
                                                    const long* __restrict__ labels,
                                                    bf16_t* __restrict__ dlogits,
                                                    float* __restrict__ loss_rows, int V,
                                                    float smoothing, float grad_scale,
                                                    long ignore_index, long tm_b) {
  __shared__ float scratch[16];
  const long row = blockIdx.x;
  const bf16_t* lr = logits + row * V;
  const long lab = labels[tm_index(row, gridDim.x, tm_b)];
  const bool ign = lab == ignore_index;
  // pass 1: online max / sum-exp, vectorized 8-wide when aligned
  float m = -INFINITY, s = 0.f, sum_logit = 0.f;
  const bool vec = (V % 8) == 0;
  if (vec) {
    for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
      const uint4 u = *(const uint4*)(lr + c);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float a = __uint_as_float(w[k] << 16), b = __uint_as_float(w[k] & 0xffff0000u);
        sum_logit += a + b;
        const float mn = fmaxf(m, fmaxf(a, b));
        s = s * __expf(m - mn) + __expf(a - mn) + __expf(b - mn);
        m = mn;
      }
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) {
      const float a = bf2f(lr[c]);
      sum_logit += a;
      const float mn = fmaxf(m, a);
      s = s * __expf(m - mn) + __expf(a - mn);
      m = mn;
    }
  }
  const float M = block_max(m, scratch);
  float sc = (m == -INFINITY) ? 0.f : s * __expf(m - M);
  const float S = block_sum(sc, scratch);
  const float SL = block_sum(sum_logit, scratch);
  const float lse = M + __logf(S);
  if (threadIdx.x == 0) {
    float loss = 0.f;
    if (!ign) {
      const float lt = bf2f(lr[lab]);
      loss = (1.f - smoothing) * (lse - lt) + smoothing * (lse - SL / V);
    }
    loss_rows[row] = loss;
  }
  if (!dlogits) return;
  bf16_t* dr = dlogits + row * V;
  const float inv = 1.f / S;
  const float eps_v = smoothing / V;
  if (vec) {
    for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
      const uint4 u = *(const uint4*)(lr + c);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c0 = c + 2 * k;
        float a = __expf(__uint_as_float(w[k] << 16) - M) * inv - eps_v;
        float b = __expf(__uint_as_float(w[k] & 0xffff0000u) - M) * inv - eps_v;
        if (c0 == lab) a -= 1.f - smoothing;
        if (c0 + 1 == lab) b -= 1.f - smoothing;
        if (ign) { a = 0.f; b = 0.f; }
        o[k] = pack_bf2(a * grad_scale, b * grad_scale);
      }
      *(uint4*)(dr + c) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) {
      float a = __expf(bf2f(lr[c]) - M) * inv - eps_v;
      if (c == lab) a -= 1.f - smoothing;
      if (ign) a = 0.f;
      dr[c] = f2bf(a * grad_scale);
    }
  }
}

void softmax_xent(const bf16_t* logits, const long* labels, bf16_t* dlogits, float* loss_rows,
                  long rows, int V, float smoothing, float grad_scale, long ignore_index,
                  hipStream_t s, long tm_b) {
  hipLaunchKernelGGL(xent_kernel, dim3(rows), dim3(256), 0, s, logits, labels, dlogits, loss_rows,
                     V, smoothing, grad_scale, ignore_index, tm_b);
}

// out[0] = scale * sum(x[0..n)): the mean loss from the per-row losses, one
// block (no torch reduce + scale kernels in the step)
__global__ void __launch_bounds__(256) sum_scale_kernel(const float* __restrict__ x, long n,
                                                        float* __restrict__ out, float scale) {
  __shared__ float scratch[16];
  float acc = 0.f;
  for (long i = threadIdx.x; i < n; i += 256) acc += x[i];
  const float t = block_sum(acc, scratch);
  if (threadIdx.x == 0) out[0] = t * scale;
}
void sum_scale(const float* x, long n, float* out, float scale, hipStream_t s) {
  hipLaunchKernelGGL(sum_scale_kernel, dim3(1), dim3(256), 0, s, x, n, out, scale);
}

// ------------------------------------------------------------------ embedding
// out[t][:] = table[ids[t]][:] * scale  (D % 8 == 0), 16 B per lane
// ids outside [0, V) (a batch built for another vocabulary) read as zero
// rows and take no gradient, instead of faulting the device
// tm_b > 0: output rows time-major (t = s * tm_b + b) from [tm_b][S] ids;
// pos (optional, [S][D]): + pos[s] after the scale (a positional table added
// in the same pass, no broadcast copy); S = pos_rows
__global__ void embed_fwd_kernel(const bf16_t* __restrict__ table, const long* __restrict__ ids,
                                 bf16_t* __restrict__ out, long T, int D, float scale, long V, long tm_b,
                                 const bf16_t* __restrict__ pos, long pos_rows) {
  const int d8 = D / 8;
  const long total = T * d8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long t = i / d8;
    const int c = (int)(i % d8) * 8;
    const long id = ids[tm_index(t, T, tm_b)];
    const uint4 u = (unsigned long)id < (unsigned long)V ? *(const uint4*)(table + id * D + c)
                                                          : make_uint4(0u, 0u, 0u, 0u);
    if (scale == 1.f && !pos) {
      *(uint4*)(out + t * D + c) = u;
    } else {
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
      uint4 pv = make_uint4(0u, 0u, 0u, 0u);
      if (pos) pv = *(const uint4*)(pos + (tm_b > 0 ? t / tm_b : t % pos_rows) * D + c);
      const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        o[k] = pack_bf2(__uint_as_float(w[k] << 16) * scale + __uint_as_float(pw[k] << 16),
                        __uint_as_float(w[k] & 0xffff0000u) * scale + __uint_as_float(pw[k] & 0xffff0000u));
      *(uint4*)(out + t * D + c) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
}
// grad_table[ids[t]] += dout[t] * scale  (fp32 atomics; rows of D contiguous)
__global__ void embed_bwd_kernel(const bf16_t* __restrict__ dout, const long* __restrict__ ids,
                                 float* __restrict__ gtable, long T, int D, float scale, long V, long tm_b) {
  const long total = T * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long t = i / D;
    const int c = (int)(i % D);
    const long id = ids[tm_index(t, T, tm_b)];
    if ((unsigned long)id < (unsigned long)V) atomicAdd(gtable + id * D + c, bf2f(dout[i]) * scale);
  }
}
void embedding_forward(const bf16_t* table, const long* ids, bf16_t* out, long T, int D,
                       float scale, hipStream_t s, long V, long tm_b, const bf16_t* pos, long pos_rows) {
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(grid_cap(T * D / 8)), dim3(256), 0, s, table, ids, out,
                     T, D, scale, V, tm_b, pos, pos_rows);
}
void embedding_backward(const bf16_t* dout, const long* ids, float* gtable, long T, int D,
                        float scale, hipStream_t s, long V, long tm_b) {
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(grid_cap(T * D)), dim3(256), 0, s, dout, ids, gtable, T,
                     D, scale, V, tm_b);
}

// ------------------------------------------------------------- column sums
// out[c] (+)= sum_r x[r][c] (bias gradients), fp32 accumulate, relu-mask opt.
__global__ void colsum_kernel(const bf16_t* __restrict__ x, float* __restrict__ out, long R, int C,
                              long rows_per_block) {
  // scalar path for C % 8 != 0
  const long r0 = blockIdx.y * rows_per_block;
  const long r1 = min(R, r0 + rows_per_block);
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    float s = 0.f;
    for (long r = r0; r < r1; ++r) s += bf2f(x[r * C + c]);
    atomicAdd(out + c, s);
  }
}

// C % 8 == 0: block = (row lane rl, 8-column group cg) over a <=2048-column
// chunk, 16 B loads, LDS combine over row lanes; block (x, y) either adds its
// column sums straight into `out` (no-return fp32 atomics, one per column per
// block: a few hundred blocks never contend measurably) or, with out ==
// nullptr, writes partial row y for col_reduce_acc.
__global__ void __launch_bounds__(256) colsum8_kernel(const bf16_t* __restrict__ x,
                                                       float* __restrict__ part, long R, int C,
                                                       long rows_per_block,
                                                       float* __restrict__ out) {
  __shared__ float red[256 * 8];
  const int c0 = blockIdx.x * 2048;
  const int cw = min(2048, C - c0);
  const int tpr = cw / 8 < 256 ? cw / 8 : 256;
  const int rpp = 256 / tpr;
  const int cg = threadIdx.x % tpr, rl = threadIdx.x / tpr;
  const long r0 = blockIdx.y * rows_per_block;
  const long r1 = min(R, r0 + rows_per_block);
  for (int cb = 0; cb < cw; cb += tpr * 8) {
    const int c = c0 + cb + cg * 8;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (rl < rpp && c < c0 + cw) {
      long r = r0 + rl;
      for (; r + 3 * rpp < r1; r += 4 * rpp) {     // 4 independent loads in flight
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *(const uint4*)(x + (r + u * rpp) * C + c);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            s[2 * k] += __uint_as_float(w[k] << 16);
            s[2 * k + 1] += __uint_as_float(w[k] & 0xffff0000u);
          }
        }
      }
      for (; r < r1; r += rpp) {
        const uint4 v = *(const uint4*)(x + r * C + c);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          s[2 * k] += __uint_as_float(w[k] << 16);
          s[2 * k + 1] += __uint_as_float(w[k] & 0xffff0000u);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) red[threadIdx.x * 8 + k] = s[k];
    __syncthreads();
    if (rl == 0 && c < c0 + cw) {
      for (int j = 1; j < rpp; ++j)
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] += red[(j * tpr + cg) * 8 + k];
      if (out) {
#pragma unroll
        for (int k = 0; k < 8; ++k) atomicAdd(out + c + k, s[k]);
      } else {
        float* pr = part + (long)blockIdx.y * C + c;
        *(float4*)pr = make_float4(s[0], s[1], s[2], s[3]);
        *(float4*)(pr + 4) = make_float4(s[4], s[5], s[6], s[7]);
      }
    }
    __syncthreads();
  }
}

// 0 (default): tiny matrices (R*C <= COLSUM_ATOMIC_MAX) in ONE launch --
// <= 64 row blocks add their column sums straight into out (fp32 atomics),
// the rest as partial rows + column reduce; 1: always partial rows; 2:
// always atomics. Measured (tools/ab_colsum.py, profiles/r3/s3/ab_colsum.json):
// atomics 3.4 vs 5.1 us at 64x1000 but 15 vs 5 us at 4096x512 and 2-3x
// slower on every larger shape
static int g_colsum = [] {
  const char* e = getenv("TAM_COLSUM");
  return e ? atoi(e) : 0;
}();
TAM_KNOB(g_colsum)
void colsum_policy(int p) { g_colsum = p; }
constexpr long COLSUM_ATOMIC_MAX = 1L << 17;

void colsum(const bf16_t* x, float* out, float* ws, long R, int C, hipStream_t s) {
  if (C % 8 == 0) {
    const int bx = (C + 2047) / 2048;
    if (g_colsum == 2 || (g_colsum == 0 && R * C <= COLSUM_ATOMIC_MAX)) {
      long rpb = (R + 63) / 64;
      if (rpb < 32) rpb = 32;
      const long by = (R + rpb - 1) / rpb;
      hipLaunchKernelGGL(colsum8_kernel, dim3(bx, by), dim3(256), 0, s, x, (float*)nullptr, R, C, rpb, out);
      return;
    }
    // >= ~512 blocks in flight, >= 32 rows each, <= COLSUM_MAX_BLOCKS partial rows
    long by = (512 + bx - 1) / bx;
    if (by > COLSUM_MAX_BLOCKS) by = COLSUM_MAX_BLOCKS;
    long rpb = (R + by - 1) / by;
    if (rpb < 32) rpb = 32;
    by = (R + rpb - 1) / rpb;
    // large matrices: partial rows + a column reduce. Straight fp32 atomics
    // from the hundreds of blocks the bandwidth needs measured slower — they
    // serialise on the same few cache lines at the memory side (VGG conv
    // bias, 64 columns: +20 us per call)
    hipLaunchKernelGGL(colsum8_kernel, dim3(bx, by), dim3(256), 0, s, x, ws, R, C, rpb,
                       (float*)nullptr);
    col_reduce_acc(ws, (int)by, C, out, out, C, s);
    return;
  }
  const int bx = (C + 255) / 256;
  long rpb = 64;
  long by = (R + rpb - 1) / rpb;
  if (by * bx > 4096) { by = 4096 / bx; if (by < 1) by = 1; rpb = (R + by - 1) / by; by = (R + rpb - 1) / rpb; }
  hipLaunchKernelGGL(colsum_kernel, dim3(bx, by), dim3(256), 0, s, x, out, R, C, rpb);
}

// ---------------------------------------------------------------- elementwise
// y = relu(x) ; dx = dy * (y > 0); y = a + b ; fp32 -> bf16 cast
__global__ void relu_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                bf16_t* __restrict__ dx, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dx[i] = bf2f(y[i]) > 0.f ? dy[i] : (bf16_t)0;
}
__global__ void relu_bwd8_kernel(const uint4* __restrict__ dy, const uint4* __restrict__ y,
                                 uint4* __restrict__ dx, long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const uint4 d = dy[i], v = y[i];
    const uint32_t wd[4] = {d.x, d.y, d.z, d.w}, wy[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t lo = (int16_t)(wy[k] & 0xffffu) > 0 ? 0x0000ffffu : 0u;   // bf16 > 0 <=> int16 > 0
      const uint32_t hi = (int32_t)(wy[k] & 0xffff0000u) > 0 ? 0xffff0000u : 0u;
      o[k] = wd[k] & (lo | hi);
    }
    dx[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}
void relu_backward(const bf16_t* dy, const bf16_t* y, bf16_t* dx, long n, hipStream_t s) {
  if (n % 8 == 0) {
    hipLaunchKernelGGL(relu_bwd8_kernel, dim3(grid_cap(n / 8)), dim3(256), 0, s, (const uint4*)dy,
                       (const uint4*)y, (uint4*)dx, n / 8);
    return;
  }
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(grid_cap(n)), dim3(256), 0, s, dy, y, dx, n);
}

__global__ void add_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                           bf16_t* __restrict__ y, long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const uint4 u = ((const uint4*)a)[i], v = ((const uint4*)b)[i];
    const uint32_t wa[4] = {u.x, u.y, u.z, u.w}, wb[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      o[k] = pack_bf2(__uint_as_float(wa[k] << 16) + __uint_as_float(wb[k] << 16),
                      __uint_as_float(wa[k] & 0xffff0000u) + __uint_as_float(wb[k] & 0xffff0000u));
    ((uint4*)y)[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}
void add_bf16(const bf16_t* a, const bf16_t* b, bf16_t* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(add_kernel, dim3(grid_cap(n / 8)), dim3(256), 0, s, a, b, y, n / 8);
}

// ---------------------------------------------------- row-block copies / sums
// Up to 4 jobs in one launch (blockIdx.y = job): out[r][0..C) = sum of the
// job's n_in inputs' rows r, every operand with its own row pitch (16-B
// aligned rows, C % 8 == 0). A last-dim concat is one job per part (n_in =
// 1, out = the part's column slice); a gradient fan-in is one job of n_in
// inputs -- the pitched column slices a concat's backward hands out.
__global__ void __launch_bounds__(256) rows_sum_kernel(RowJobs jb, long R) {
  const RowJob& j = jb.job[blockIdx.y];
  const int c8 = j.C / 8;
  const long total = R * c8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / c8;
    const int c = (int)(i % c8) * 8;
    uint4 u = *(const uint4*)(j.in[0] + r * j.ld_in[0] + c);
    if (j.n_in > 1) {
      float f[8];
      const uint32_t* w = (const uint32_t*)&u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        f[2 * k] = __uint_as_float(w[k] << 16);
        f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
      }
      for (int q = 1; q < j.n_in; ++q) {
        const uint4 v = *(const uint4*)(j.in[q] + r * j.ld_in[q] + c);
        const uint32_t* x = (const uint32_t*)&v;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          f[2 * k] += __uint_as_float(x[k] << 16);
          f[2 * k + 1] += __uint_as_float(x[k] & 0xffff0000u);
        }
      }
      u = make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
    }
    *(uint4*)(j.out + r * j.ld_out + c) = u;
  }
}
void rows_sum(const RowJobs& jb, int njobs, long R, hipStream_t s) {
  long mx = 0;
  for (int q = 0; q < njobs; ++q) mx = std::max(mx, R * (jb.job[q].C / 8));
  hipLaunchKernelGGL(rows_sum_kernel, dim3(grid_cap(mx), njobs), dim3(256), 0, s, jb, R);
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}
void cast_f32_bf16(const float* x, bf16_t* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_cap(n)), dim3(256), 0, s, x, y, n);
}

}  // namespace tam
