// tiresias_amd — shared device helpers for the CDNA4 (gfx950) kernel library.
//
// Everything here is written for MI355X only: 64-lane wavefronts, MFMA bf16
// fragments, 16-byte vector memory ops. No CUDA / dual-platform paths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace tam {

typedef unsigned short bf16_t;  // raw bf16 bits in memory
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;

// shards of a BatchNorm statistics accumulator (fp64 [BN_SHARDS][2C], see
// norm.hip "BN sums"): conv epilogues spread their atomics over them
constexpr int BN_SHARDS = 16;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// round-to-nearest-even fp32 -> bf16 (NaN -> quiet NaN): gfx950's hardware
// conversion, one v_cvt_pk_bf16_f32 per PAIR of values (the bit-twiddling RNE
// it replaces was ~7 VALU per value, most of a store epilogue's VALU)
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64, up to 1024 threads.
// `scratch` must hold >= 16 floats in LDS.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}

__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, scratch[i]);
  return r;
}

// Bijective XCD-aware remap of a linear workgroup id (8 XCDs, private L2s):
// consecutive logical tiles land on the same XCD so neighbouring tiles share
// operand panels in one L2 (guide §5.5 T1, bijective form for nwg % 8 != 0).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int xcd = orig & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

// Zero `bytes` at `p` on stream `s` with a kernel (16-B vector stores).
// Used instead of hipMemsetAsync everywhere on the compute path: memset
// nodes in replayed hipGraphs were measured to race with the kernel nodes
// that follow them (ResNet-50 loss diverged only under graph replay with the
// device idle between steps); a kernel node is ordered like any other.
void zero_async(void* p, size_t bytes, hipStream_t s);
// rows x cols fp32 block with row pitch ld (floats)
void zero_async_2d(float* p, long ld, int cols, int rows, hipStream_t s);

// ---- host-side registry of the library's tuning knobs (every *_policy /
// *_force setting): tests snapshot it at load and restore it after each test
// (ops.cpp policy_state / policy_load), so no test leaves a non-production
// configuration behind for the next one
struct KnobRef {
  const char* name;
  int* p;
};
inline std::vector<KnobRef>& knob_registry() {
  static std::vector<KnobRef> v;
  return v;
}
struct KnobReg {
  KnobReg(const char* n, int* p) { knob_registry().push_back({n, p}); }
};
#define TAM_KNOB(var) static ::tam::KnobReg var##_knob_reg_(#var, &var);

}  // namespace tam

#define TAM_HIP_CHECK(expr)                                                    \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e),        \
              __FILE__, __LINE__);                                             \
      abort();                                                                 \
    }                                                                          \
  } while (0)
