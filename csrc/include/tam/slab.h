// fp32 split-K slab reduction shared by the conv weight-gradient kernels
// (conv_dma.h DMA wgrad, conv_stem.hip stem wgrad).
#pragma once
#include <hip/hip_runtime.h>

#include "tam/common.h"

namespace tam {

// dw[i] = (mode ? dw[i] : 0) + sum_z ws[z][i] over mn contiguous floats (mn % 4
// == 0). A block is (256 / L) float4 columns x L split lanes: every thread
// sums a strided subset of the slabs with independent loads, the lanes meet
// in LDS. L grows with the split count so no thread walks a long dependent
// chain of slab loads (a one-thread-per-element reduce over 98 slabs of a
// 64K-float dW measured 12 us slower than the atomics it replaced).
static __global__ void __launch_bounds__(256) wg_slab_reduce_kernel(const float* __restrict__ ws, int sp, long mn,
                                                                    float* __restrict__ dw, int mode, int L) {
  __shared__ f32x4_t red[256];
  const int cols = 256 / L;
  const int cx = threadIdx.x % cols, zy = threadIdx.x / cols;
  const long n4 = mn >> 2;
  const long i = (long)blockIdx.x * cols + cx;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  if (i < n4) {
    const f32x4_t* w4 = (const f32x4_t*)ws + i;
    const long zs = n4 * L;
    int z = zy;
    for (; z + 3 * L < sp; z += 4 * L) {
      const f32x4_t v0 = w4[z * n4], v1 = w4[z * n4 + zs], v2 = w4[z * n4 + 2 * zs], v3 = w4[z * n4 + 3 * zs];
      acc += (v0 + v1) + (v2 + v3);
    }
    for (; z < sp; z += L) acc += w4[z * n4];
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (zy == 0 && i < n4) {
    for (int k = 1; k < L; ++k) acc += red[k * cols + cx];
    f32x4_t* o = (f32x4_t*)dw + i;
    *o = mode ? *o + acc : acc;
  }
}

inline void wgrad_slab_reduce(const float* ws, int sp, long mn, float* dw, int mode, hipStream_t s) {
  int L = 1;
  while (L < 64 && (sp + L - 1) / L > 8) L *= 2;   // <= 8 slab loads per thread
  const int cols = 256 / L;
  const long blocks = ((mn >> 2) + cols - 1) / cols;
  hipLaunchKernelGGL(wg_slab_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ws, sp, mn, dw, mode, L);
}

}  // namespace tam
