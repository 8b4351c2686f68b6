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

// Many slab reduces in ONE launch (the deferred conv weight-gradient slabs
// of a backward): blocks [b0_e, b0_{e+1}) serve entry e exactly as
// wg_slab_reduce_kernel would for that entry alone.
constexpr int SLAB_BATCH_MAX = 40;
struct SlabBatch {
  const float* ws[SLAB_BATCH_MAX];
  float* dw[SLAB_BATCH_MAX];
  long mn[SLAB_BATCH_MAX];
  int sp[SLAB_BATCH_MAX], mode[SLAB_BATCH_MAX], L[SLAB_BATCH_MAX], b0[SLAB_BATCH_MAX + 1];
  int n;
};

static __global__ void __launch_bounds__(256) wg_slab_reduce_batch_kernel(SlabBatch b) {
  __shared__ f32x4_t red[256];
  int e = 0;
  while (e + 1 < b.n && (int)blockIdx.x >= b.b0[e + 1]) ++e;
  const int L = b.L[e], sp = b.sp[e];
  const int cols = 256 / L;
  const int cx = threadIdx.x % cols, zy = threadIdx.x / cols;
  const long n4 = b.mn[e] >> 2;
  const long i = (long)((int)blockIdx.x - b.b0[e]) * cols + cx;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  if (i < n4) {
    const f32x4_t* w4 = (const f32x4_t*)b.ws[e] + i;
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
    f32x4_t* o = (f32x4_t*)b.dw[e] + i;
    *o = b.mode[e] ? *o + acc : acc;
  }
}

inline int wgrad_slab_lanes(int sp) {
  int L = 1;
  while (L < 64 && (sp + L - 1) / L > 8) L *= 2;   // <= 8 slab loads per thread
  return L;
}

inline void wgrad_slab_reduce_batch(const float* const* ws, const int* sp, const long* mn, float* const* dw,
                                    const int* mode, int n, hipStream_t s) {
  for (int base = 0; base < n; base += SLAB_BATCH_MAX) {
    SlabBatch b{};
    const int m = n - base < SLAB_BATCH_MAX ? n - base : SLAB_BATCH_MAX;
    int blocks = 0;
    for (int i = 0; i < m; ++i) {
      const int j = base + i;
      b.ws[i] = ws[j]; b.dw[i] = dw[j]; b.mn[i] = mn[j]; b.sp[i] = sp[j]; b.mode[i] = mode[j];
      b.L[i] = wgrad_slab_lanes(sp[j]);
      b.b0[i] = blocks;
      const int cols = 256 / b.L[i];
      blocks += (int)(((mn[j] >> 2) + cols - 1) / cols);
    }
    b.b0[m] = blocks;
    b.n = m;
    if (blocks) hipLaunchKernelGGL(wg_slab_reduce_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, s, b);
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
