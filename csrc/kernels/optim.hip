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
#include "tam/common.h"
#include "tam/kernels.h"

namespace tam {

__global__ void __launch_bounds__(256) sgd_kernel(float* __restrict__ w, float* __restrict__ g,
                                                   float* __restrict__ mom,
                                                   bf16_t* __restrict__ wb, long n4, float lr,
                                                   float momentum, float wd, float gscale,
                                                   int nesterov, int zero_grad, const unsigned* guard) {
  if (guard != nullptr && *guard != 0u) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
      ((float4*)g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float4 wv = ((float4*)w)[i];
    float4 gv = ((float4*)g)[i];
    float4 mv = ((float4*)mom)[i];
    float* wp = (float*)&wv; float* gp = (float*)&gv; float* mp = (float*)&mv;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float d = gp[k] * gscale + wd * wp[k];
      mp[k] = momentum * mp[k] + d;
      d = nesterov ? d + momentum * mp[k] : mp[k];
      wp[k] -= lr * d;
    }
    ((float4*)w)[i] = wv;
    ((float4*)mom)[i] = mv;
    if (zero_grad) ((float4*)g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    ((uint2*)wb)[i] = make_uint2(pack_bf2(wp[0], wp[1]), pack_bf2(wp[2], wp[3]));
  }
}

__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ w, float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    bf16_t* __restrict__ wb, long n4, float lr,
                                                    float b1, float b2, float eps, float wd,
                                                    float bc1, float bc2, float gscale,
                                                    int zero_grad, const unsigned* guard) {
  if (guard != nullptr && *guard != 0u) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
      ((float4*)g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float4 wv = ((float4*)w)[i], gv = ((float4*)g)[i], mv = ((float4*)m)[i], vv = ((float4*)v)[i];
    float* wp = (float*)&wv; float* gp = (float*)&gv; float* mp = (float*)&mv; float* vp = (float*)&vv;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gr = gp[k] * gscale;
      mp[k] = b1 * mp[k] + (1.f - b1) * gr;
      vp[k] = b2 * vp[k] + (1.f - b2) * gr * gr;
      const float mh = mp[k] / bc1, vh = vp[k] / bc2;
      wp[k] -= lr * (mh / (sqrtf(vh) + eps) + wd * wp[k]);   // decoupled (AdamW)
    }
    ((float4*)w)[i] = wv; ((float4*)m)[i] = mv; ((float4*)v)[i] = vv;
    if (zero_grad) ((float4*)g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    ((uint2*)wb)[i] = make_uint2(pack_bf2(wp[0], wp[1]), pack_bf2(wp[2], wp[3]));
  }
}

static int ogrid(long n4) {
  long b = (n4 + 255) / 256;
  if (b > 4096) b = 4096;
  return (int)(b < 1 ? 1 : b);
}

void sgd_step(float* w, float* g, float* mom, bf16_t* wb, long n, float lr, float momentum,
              float wd, float gscale, int nesterov, int zero_grad, hipStream_t s, const unsigned* guard) {
  // n % 4 == 0 (arena segments are padded to 64 elements)
  hipLaunchKernelGGL(sgd_kernel, dim3(ogrid(n / 4)), dim3(256), 0, s, w, g, mom, wb, n / 4, lr,
                     momentum, wd, gscale, nesterov, zero_grad, guard);
}

void adam_step(float* w, float* g, float* m, float* v, bf16_t* wb, long n, float lr, float b1,
               float b2, float eps, float wd, int step, float gscale, int zero_grad,
               hipStream_t s, const unsigned* guard) {
  const float bc1 = 1.f - powf(b1, (float)step), bc2 = 1.f - powf(b2, (float)step);
  hipLaunchKernelGGL(adam_kernel, dim3(ogrid(n / 4)), dim3(256), 0, s, w, g, m, v, wb, n / 4, lr,
                     b1, b2, eps, wd, bc1, bc2, gscale, zero_grad, guard);
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
