// tiresias_amd — fused optimizer steps over a job's *flat* parameter arena.
//
// Every job keeps its parameters in one contiguous fp32 master buffer with a
// bf16 shadow (the compute copy the kernels read), one fp32 gradient buffer
// (what the bucketed RCCL all-reduce reduces in place) and its optimizer
// state. One launch updates the whole model: read grad + master + state,
// write master + state + bf16 shadow, and zero the gradient for the next
// iteration (saves the separate memset pass). 16 B per lane.
//
// ``guard`` (nullable): a device word that, when non-zero, turns the step
// into a gradient reset only -- no master / state / shadow update. The
// trainer of a GNMT job passes ITS OWN persistent-LSTM timeout word
// (models/gnmt.py GNMT.err[0], bumped by a timed-out grid barrier of that
// job only): a step whose recurrence read h / dG that had not arrived must
// not reach the weights. lstm_guard_step then moves the word into the job's
// skipped-step count (err[1]), which the worker subtracts from the round's
// progress and uses to switch the job to the per-step recurrence.
#include <cstdlib>

#include "tam/common.h"
#include "tam/kernels.h"

namespace tam {

__global__ void __launch_bounds__(256) sgd_kernel(float* __restrict__ w, float* __restrict__ g,
                                                   float* __restrict__ mom,
                                                   bf16_t* __restrict__ wb, long n4, float lr,
                                                   float momentum, float wd0, float gscale,
                                                   int nesterov, int zero_grad, const unsigned* guard,
                                                   long zero_from4, long wd_until4) {
  if (guard != nullptr && *guard != 0u) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
      if (i >= zero_from4) ((float4*)g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float4 wv = ((float4*)w)[i];
    float4 gv = ((float4*)g)[i];
    float4 mv = ((float4*)mom)[i];
    float* wp = (float*)&wv; float* gp = (float*)&gv; float* mp = (float*)&mv;
    const float wd = i < wd_until4 ? wd0 : 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float d = __builtin_fmaf(wd, wp[k], gp[k] * gscale);
      mp[k] = __builtin_fmaf(momentum, mp[k], d);
      d = nesterov ? __builtin_fmaf(momentum, mp[k], d) : mp[k];
      wp[k] = __builtin_fmaf(-lr, d, wp[k]);
    }
    ((float4*)w)[i] = wv;
    ((float4*)mom)[i] = mv;
    if (zero_grad && i >= zero_from4) ((float4*)g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    ((uint2*)wb)[i] = make_uint2(pack_bf2(wp[0], wp[1]), pack_bf2(wp[2], wp[3]));
  }
}

__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ w, float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    bf16_t* __restrict__ wb, long n4, float lr,
                                                    float b1, float b2, float eps, float wd0,
                                                    float bc1, float bc2, float gscale,
                                                    int zero_grad, const unsigned* guard, long zero_from4,
                                                    long wd_until4) {
  if (guard != nullptr && *guard != 0u) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
      if (i >= zero_from4) ((float4*)g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const float ib1 = 1.f / bc1, ib2 = 1.f / bc2;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float4 wv = ((float4*)w)[i], gv = ((float4*)g)[i], mv = ((float4*)m)[i], vv = ((float4*)v)[i];
    float* wp = (float*)&wv; float* gp = (float*)&gv; float* mp = (float*)&mv; float* vp = (float*)&vv;
    const float wd = i < wd_until4 ? wd0 : 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gr = gp[k] * gscale;
      mp[k] = __builtin_fmaf(b1, mp[k], (1.f - b1) * gr);
      vp[k] = __builtin_fmaf(b2, vp[k], (1.f - b2) * gr * gr);
      const float mh = mp[k] * ib1, vh = vp[k] * ib2;
      const float u = __builtin_fmaf(wd, wp[k], mh / (sqrtf(vh) + eps));   // decoupled (AdamW)
      wp[k] = __builtin_fmaf(-lr, u, wp[k]);
    }
    ((float4*)w)[i] = wv; ((float4*)m)[i] = mv; ((float4*)v)[i] = vv;
    if (zero_grad && i >= zero_from4) ((float4*)g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    ((uint2*)wb)[i] = make_uint2(pack_bf2(wp[0], wp[1]), pack_bf2(wp[2], wp[3]));
  }
}

// Every form spells its arithmetic as explicit FMAs: the element update is
// then one fixed rounding sequence whichever path (kernel, unrolled group or
// tail) covers the element, so a step is bitwise independent of the grid,
// the variant and how an arena is split into launches (contraction was left
// to the compiler before and differed between the unrolled and tail bodies).
// Streaming variants (optim_variant): U float4 groups per thread per
// iteration, all loads issued before any math (U x 4 x 16 B in flight per
// lane), NT: non-temporal loads / stores (every byte is touched once per
// step; keeps the step from evicting the next forward's L2 / MALL working
// set). Tail groups (n4 % U) are handled with the same body at U = 1.
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
template <int U, bool NT>
__device__ __forceinline__ float4 ld4(const float* p, long i) {
  if constexpr (NT) {
    const f32x4_t r = __builtin_nontemporal_load((const f32x4_t*)p + i);
    return make_float4(r[0], r[1], r[2], r[3]);
  } else {
    return ((const float4*)p)[i];
  }
}
template <bool NT>
__device__ __forceinline__ void st4(float* p, long i, float4 v) {
  if constexpr (NT) __builtin_nontemporal_store(f32x4_t{v.x, v.y, v.z, v.w}, (f32x4_t*)p + i);
  else ((float4*)p)[i] = v;
}
template <bool NT>
__device__ __forceinline__ void st2(bf16_t* p, long i, uint2 v) {
  if constexpr (NT) __builtin_nontemporal_store(u32x2_t{v.x, v.y}, (u32x2_t*)p + i);
  else ((uint2*)p)[i] = v;
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) adam_stream_kernel(float* __restrict__ w, float* __restrict__ g,
                                                           float* __restrict__ m, float* __restrict__ v,
                                                           bf16_t* __restrict__ wb, long n4, float lr, float b1,
                                                           float b2, float eps, float wd0, float bc1, float bc2,
                                                           float gscale, int zero_grad, const unsigned* guard,
                                                           long zero_from4, long wd_until4) {
  const long stride = (long)gridDim.x * blockDim.x;
  if (guard != nullptr && *guard != 0u) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride)
      if (i >= zero_from4) st4<NT>(g, i, make_float4(0.f, 0.f, 0.f, 0.f));
    return;
  }
  const float ib1 = 1.f / bc1, ib2 = 1.f / bc2;
  auto body = [&](long i, float4 wv, float4 gv, float4 mv, float4 vv) {
    float* wp = (float*)&wv; float* gp = (float*)&gv; float* mp = (float*)&mv; float* vp = (float*)&vv;
    const float wd = i < wd_until4 ? wd0 : 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gr = gp[k] * gscale;
      mp[k] = __builtin_fmaf(b1, mp[k], (1.f - b1) * gr);
      vp[k] = __builtin_fmaf(b2, vp[k], (1.f - b2) * gr * gr);
      const float mh = mp[k] * ib1, vh = vp[k] * ib2;
      const float u = __builtin_fmaf(wd, wp[k], mh / (sqrtf(vh) + eps));   // decoupled (AdamW)
      wp[k] = __builtin_fmaf(-lr, u, wp[k]);
    }
    st4<NT>(w, i, wv); st4<NT>(m, i, mv); st4<NT>(v, i, vv);
    if (zero_grad && i >= zero_from4) st4<NT>(g, i, make_float4(0.f, 0.f, 0.f, 0.f));
    st2<NT>(wb, i, make_uint2(pack_bf2(wp[0], wp[1]), pack_bf2(wp[2], wp[3])));
  };
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long full = n4 / (U * stride) * (U * stride);
  for (long base = t; base < full; base += U * stride) {
    float4 wv[U], gv[U], mv[U], vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + u * stride;
      wv[u] = ld4<U, NT>(w, i); gv[u] = ld4<U, NT>(g, i); mv[u] = ld4<U, NT>(m, i); vv[u] = ld4<U, NT>(v, i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) body(base + u * stride, wv[u], gv[u], mv[u], vv[u]);
  }
  for (long i = full + t; i < n4; i += stride)
    body(i, ld4<1, NT>(w, i), ld4<1, NT>(g, i), ld4<1, NT>(m, i), ld4<1, NT>(v, i));
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) sgd_stream_kernel(float* __restrict__ w, float* __restrict__ g,
                                                          float* __restrict__ mom, bf16_t* __restrict__ wb, long n4,
                                                          float lr, float momentum, float wd0, float gscale,
                                                          int nesterov, int zero_grad, const unsigned* guard,
                                                          long zero_from4, long wd_until4) {
  const long stride = (long)gridDim.x * blockDim.x;
  if (guard != nullptr && *guard != 0u) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride)
      if (i >= zero_from4) st4<NT>(g, i, make_float4(0.f, 0.f, 0.f, 0.f));
    return;
  }
  auto body = [&](long i, float4 wv, float4 gv, float4 mv) {
    float* wp = (float*)&wv; float* gp = (float*)&gv; float* mp = (float*)&mv;
    const float wd = i < wd_until4 ? wd0 : 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float d = __builtin_fmaf(wd, wp[k], gp[k] * gscale);
      mp[k] = __builtin_fmaf(momentum, mp[k], d);
      d = nesterov ? __builtin_fmaf(momentum, mp[k], d) : mp[k];
      wp[k] = __builtin_fmaf(-lr, d, wp[k]);
    }
    st4<NT>(w, i, wv); st4<NT>(mom, i, mv);
    if (zero_grad && i >= zero_from4) st4<NT>(g, i, make_float4(0.f, 0.f, 0.f, 0.f));
    st2<NT>(wb, i, make_uint2(pack_bf2(wp[0], wp[1]), pack_bf2(wp[2], wp[3])));
  };
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long full = n4 / (U * stride) * (U * stride);
  for (long base = t; base < full; base += U * stride) {
    float4 wv[U], gv[U], mv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + u * stride;
      wv[u] = ld4<U, NT>(w, i); gv[u] = ld4<U, NT>(g, i); mv[u] = ld4<U, NT>(mom, i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) body(base + u * stride, wv[u], gv[u], mv[u]);
  }
  for (long i = full + t; i < n4; i += stride) body(i, ld4<1, NT>(w, i), ld4<1, NT>(g, i), ld4<1, NT>(mom, i));
}

// 0: adam_kernel / sgd_kernel (one group per thread per iteration); 3: U=4
// + NT (1 / 2, U=2 with / without NT, measured between the two and were
// dropped). -1 (default): optim_pick.
static int g_optim_variant = [] {
  const char* e = getenv("TAM_OPTIM_VARIANT");   // A/B runs
  return e ? atoi(e) : -1;
}();
TAM_KNOB(g_optim_variant)
void optim_variant(int v) { g_optim_variant = v; }
// auto: the streaming form for every arena, launched at ONE block per CU
// (ogrid). Rounds 4-5 ran it on a 4096-block grid, where its isolated gain
// on Adam did not survive inside the graph step; at one block per CU each
// CU keeps 4 waves x 16 float4 loads in flight on a single arena stream
// (fewer open DRAM pages than 16 blocks interleaving), and it wins both
// isolated and in the step. Same box (tools/bench_optim.py,
// profiles/r6/optim_grid.md):
//   isolated, us (v0 @4096 -> v3 @256): GNMT Adam 1593 -> 1393,
//   Transformer Adam 382 -> 327, VGG-16 SGD 795 -> 627, ResNet-50 SGD 120 -> 108;
//   graph step, ms: GNMT 9.73-9.75 -> 9.41-9.48, Transformer 4.95-4.96 ->
//   4.90-4.91, VGG-16 6.57-6.60 -> 6.47, ResNet-50 equal.
static int optim_pick(long, bool) {
  return g_optim_variant >= 0 ? g_optim_variant : 3;
}

// grid cap of the optimizer launches (blocks of 256; each thread strides
// over the arena); 0 (default): one block per CU. TAM_OPTIM_GRID /
// optim_grid(): A/B of the cap. Partial waves of blocks (1.5 per CU) measured
// 10-15 % slower than whole multiples.
static int g_optim_grid = [] {
  const char* e = getenv("TAM_OPTIM_GRID");
  return e ? atoi(e) : 0;
}();
TAM_KNOB(g_optim_grid)
void optim_grid(int blocks) { g_optim_grid = blocks > 0 ? blocks : 0; }

static int ogrid(long n4) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  const long cap = g_optim_grid > 0 ? g_optim_grid : cus;
  long b = (n4 + 255) / 256;
  if (b > cap) b = cap;
  return (int)(b < 1 ? 1 : b);
}

// zero_from / wd_until (elements, multiples of 4): the gradient is reset only
// from zero_from on (store-first gradients before it, Fx.grad_mode), weight
// decay applies only below wd_until -- one launch over a whole arena's
// store / decay / no-decay regions (was three launches through round 5)
void sgd_step(float* w, float* g, float* mom, bf16_t* wb, long n, float lr, float momentum,
              float wd, float gscale, int nesterov, int zero_grad, hipStream_t s, const unsigned* guard,
              long zero_from, long wd_until) {
  // n % 4 == 0 (arena segments are padded to 64 elements)
  const dim3 grid(ogrid(n / 4));
  const long zf4 = zero_from / 4, wu4 = wd_until < 0 ? n / 4 : wd_until / 4;
  switch (optim_pick(n / 4, false)) {
    case 3:
      hipLaunchKernelGGL((sgd_stream_kernel<4, true>), grid, dim3(256), 0, s, w, g, mom, wb, n / 4, lr, momentum, wd,
                         gscale, nesterov, zero_grad, guard, zf4, wu4);
      break;
    default:
      hipLaunchKernelGGL(sgd_kernel, grid, dim3(256), 0, s, w, g, mom, wb, n / 4, lr, momentum, wd, gscale, nesterov,
                         zero_grad, guard, zf4, wu4);
  }
}

void adam_step(float* w, float* g, float* m, float* v, bf16_t* wb, long n, float lr, float b1,
               float b2, float eps, float wd, int step, float gscale, int zero_grad,
               hipStream_t s, const unsigned* guard, long zero_from, long wd_until) {
  const float bc1 = 1.f - powf(b1, (float)step), bc2 = 1.f - powf(b2, (float)step);
  const dim3 grid(ogrid(n / 4));
  const long zf4 = zero_from / 4, wu4 = wd_until < 0 ? n / 4 : wd_until / 4;
  switch (optim_pick(n / 4, true)) {
    case 3:
      hipLaunchKernelGGL((adam_stream_kernel<4, true>), grid, dim3(256), 0, s, w, g, m, v, wb, n / 4, lr, b1, b2, eps,
                         wd, bc1, bc2, gscale, zero_grad, guard, zf4, wu4);
      break;
    default:
      hipLaunchKernelGGL(adam_kernel, grid, dim3(256), 0, s, w, g, m, v, wb, n / 4, lr, b1, b2, eps, wd, bc1, bc2,
                         gscale, zero_grad, guard, zf4, wu4);
  }
}

__global__ void lstm_guard_step_kernel(unsigned* err) {
  if (threadIdx.x == 0 && err[0] != 0u) {
    err[1] += 1u;
    err[0] = 0u;
  }
}

void lstm_guard_step(unsigned* err, hipStream_t s) {
  hipLaunchKernelGGL(lstm_guard_step_kernel, dim3(1), dim3(64), 0, s, err);
}

}  // namespace tam
