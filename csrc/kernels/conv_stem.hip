// ResNet stem convolution (7x7, stride 2, pad 3, 8 input channels -> 64),
// forward. SURVEY.md §2 (model zoo: ResNet-50); the reference's models are
// plain torchvision nets trained through its job wrapper
// (reference: core/models/*, driven from run_sim.py job traces).
//
// The generic paths gather 16-byte (one tap, 8 channels) rows with per-load
// index arithmetic: 143 us for batch 64 at 224x224, ~280 TF/s. Here one
// persistent block per CU walks row groups of ST_ROWS output rows:
//   * the (2 ST_ROWS + 5) input rows a group reads (zero-padded, W + 6
//     pixels wide) are DMA'd into LDS one group ahead; every A fragment is one
//     ds_read_b128 of patch[2 pr + r][2 q + s][0..7] (lane = pixel q, k-group
//     = tap), no index math beyond the tap's (r, s);
//   * all 49 taps x 64 output channels of weights live in registers as MFMA
//     B fragments (13 K-steps of 4 taps; 2 N-tiles per wave), loaded once
//     per CU, so each A fragment feeds 2 MFMAs;
//   * each 16-pixel x 64-channel output tile goes through a per-wave LDS
//     tile and leaves as 2 KiB of contiguous 16-byte stores, with bias /
//     ReLU and the BatchNorm sums of the stored values (sharded fp64, as
//     conv_dma.h) in the epilogue.
#include <hip/hip_runtime.h>

#include "tam/common.h"
#include "tam/igemm.h"
#include "tam/slab.h"

namespace tam {

constexpr int ST_ROWS = 4;                 // output rows per row group
constexpr int ST_PROWS = 2 * ST_ROWS + 5;  // input rows they read
constexpr int ST_PW_MAX = 230;             // patch width W + 6, W <= 224
constexpr int ST_PENT = 3008;              // patch entries (16 B), ST_PROWS * ST_PW_MAX in 64-entry chunks
constexpr int ST_KSTEPS = 13;              // 49 taps (+3 zero) / 4 taps per MFMA

typedef __attribute__((address_space(3))) void st_lds_void_t;
static __device__ __attribute__((aligned(64))) uint4 g_st_zero[1];   // padding source (zero-initialised)

struct StemArgs {
  const bf16_t* x;      // [N][H][W][8]
  const bf16_t* w;      // [64][7][7][8]
  bf16_t* y;            // [N][P][Q][64]
  const bf16_t* bias;   // [64] or null
  double* stats;        // [BN_SHARDS][128] (sum | sum of squares) or null
  int N, H, W, P, Q, relu, rblocks;
};

// Persistent: block b takes row groups b, b + grid, ...; the next group's
// patch is DMA'd (global_load_lds, lane-linear 16-byte entries, padding
// from a zero word) into the other buffer while the current one computes.
// 8 waves: wave w owns output channels 32 (w & 1) .. +32 (its 2 x 13 B
// fragments, 104 VGPRs) of M-tiles w/2, w/2 + 4, ...; two waves per SIMD,
// each with its 13 A fragments in flight before the MFMAs (4 N-tiles per
// wave needed 208 VGPRs of weights and serialised every LDS read).
__global__ void __launch_bounds__(512, 1) conv_stem_fwd_kernel(StemArgs a) {
  __shared__ __attribute__((aligned(1024))) uint4 patch[2][ST_PENT];
  __shared__ __attribute__((aligned(16))) bf16_t otile[8][16 * 32];
  __shared__ float red[128];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nh = wv & 1, mw = wv >> 1;
  const int pw = a.W + 6, nent = ST_PROWS * pw, nchunk = (nent + 63) / 64;
  const int ngroups = a.N * a.rblocks;
  auto stage = [&](int g, int buf) {
    const int n = g / a.rblocks, h0 = 2 * ((g - n * a.rblocks) * ST_ROWS) - 3;
    for (int ch = wv; ch < nchunk; ch += 8) {
      const int i = ch * 64 + lane;
      const int r = i / pw, c = i - r * pw;
      const int h = h0 + r, wc = c - 3;
      const void* src = (const void*)g_st_zero;
      if (i < nent && (unsigned)h < (unsigned)a.H && (unsigned)wc < (unsigned)a.W)
        src = (const void*)(a.x + (((long)n * a.H + h) * a.W + wc) * 8);
      __builtin_amdgcn_global_load_lds(src, (st_lds_void_t*)(&patch[buf][ch * 64]), 16, 0, 0);
    }
  };
  if ((int)blockIdx.x < ngroups) stage(blockIdx.x, 0);
  if (tid < 128) red[tid] = 0.f;
  // B fragments: lane -> out channel 32 nh + 16 nt + lane%16, taps 4 ks + lane/16
  const int kg = lane >> 4, col = lane & 15;
  s16x8_t bw[2][ST_KSTEPS];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ks = 0; ks < ST_KSTEPS; ++ks) {
      const int tap = ks * 4 + kg;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (tap < 49) v = *(const uint4*)(a.w + ((long)(32 * nh + nt * 16 + col) * 49 + tap) * 8);
      bw[nt][ks] = __builtin_bit_cast(s16x8_t, v);
    }
  float bv[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) bv[nt] = a.bias ? bf2f(a.bias[32 * nh + nt * 16 + col]) : 0.f;

  float ssum[2] = {0.f, 0.f}, ssq[2] = {0.f, 0.f};
  const int mtr = (a.Q + 15) / 16;
  bf16_t* ot = otile[wv];
  int it = 0;
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x, ++it) {
    const int buf = it & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA chunks (and stores) done
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                       // every wave's chunks; the other buffer is free
    asm volatile("" ::: "memory");
    if (g + (int)gridDim.x < ngroups) stage(g + gridDim.x, buf ^ 1);
    const int n = g / a.rblocks, p0 = (g - n * a.rblocks) * ST_ROWS;
    const int rows = min(ST_ROWS, a.P - p0);
    for (int t = mw; t < rows * mtr; t += 4) {
      const int pr = t / mtr, q0 = (t - pr * mtr) * 16;
      int q = q0 + col;
      q = q < a.Q ? q : a.Q - 1;                       // tail pixels: any in-patch read
      const uint4* prow = &patch[buf][(2 * pr) * pw + 2 * q];
      s16x8_t af[ST_KSTEPS];
#pragma unroll
      for (int ks = 0; ks < ST_KSTEPS; ++ks) {
        int tap = ks * 4 + kg;
        tap = tap < 49 ? tap : 48;                     // zero weights there
        const int r = tap / 7, s = tap - 7 * (tap / 7);
        af[ks] = __builtin_bit_cast(s16x8_t, prow[r * pw + s]);
      }
      f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int ks = 0; ks < ST_KSTEPS; ++ks)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[ks]),
                                                            __builtin_bit_cast(bf16x8_t, bw[nt][ks]), acc[nt], 0, 0,
                                                            0);
      // C[i][j]: pixel q0 + 4 kg + r, channel 32 nh + 16 nt + col
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[nt][r] + bv[nt];
          if (a.relu) v = fmaxf(v, 0.f);
          const bf16_t b = f2bf(v);
          const int pi = 4 * kg + r;
          ot[pi * 32 + nt * 16 + col] = b;
          if (q0 + pi < a.Q) {
            const float sv = bf2f(b);
            ssum[nt] += sv;
            ssq[nt] += sv * sv;
          }
        }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // 16 pixels x this wave's 64-byte half of each 128-byte pixel row
      bf16_t* dst = a.y + (((long)n * a.P + p0 + pr) * a.Q + q0) * 64 + 32 * nh;
      {
        const int pi = lane >> 2, part = lane & 3;
        const uint4 v = *(const uint4*)(ot + pi * 32 + part * 8);
        if (q0 + pi < a.Q) *(uint4*)(dst + pi * 64 + part * 8) = v;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (!a.stats) return;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    float s1 = ssum[nt], s2 = ssq[nt];
    s1 += __shfl_xor(s1, 16, 64); s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 16, 64); s2 += __shfl_xor(s2, 32, 64);
    if (lane < 16) {
      atomicAdd(&red[32 * nh + nt * 16 + lane], s1);
      atomicAdd(&red[64 + 32 * nh + nt * 16 + lane], s2);
    }
  }
  __syncthreads();
  if (tid < 128) unsafeAtomicAdd(a.stats + (long)(blockIdx.x % BN_SHARDS) * 128 + tid, (double)red[tid]);
}

// ---------------------------------------------------------------------------
// Stem weight gradient: dW[k][tap][c] = sum_pix dY[pix][k] X[pix @ tap][c],
// an MFMA GEMM with M = 64 output channels, N = 49 taps x 8 channels (392,
// as 25 16-column tiles of two taps each), reduction over output pixels in
// 32-pixel K-steps. Both operands are pixel-major in memory; each lane needs
// 8 consecutive pixels of one column, which ds_read_tr16_b64 delivers from
// any per-lane row addresses: A rows are dY pixels of the staged dY tile,
// B rows are the patch entries (2 pr + r, 2 q + s) of a tap -- the im2col
// matrix is never formed. Persistent blocks (one per CU) double-buffer row
// groups of ST_WROWS output rows (dY rows zero-padded to 128 pixels + their
// 2 ST_WROWS + 5 input rows), accumulate a private dW partial in registers
// and store it to an fp32 slab; one split-parallel reduce adds the slabs.
// ---------------------------------------------------------------------------
constexpr int ST_WROWS = 2;                      // output rows per group
constexpr int ST_WPROWS = 2 * ST_WROWS + 5;      // input rows they read
constexpr int ST_WPENT = 2112;                   // patch entries, ST_WPROWS * ST_PW_MAX in 64-entry chunks
constexpr int ST_WDYENT = ST_WROWS * 128 * 8;    // dY entries: rows x 128 pixels x 8 (16 B)
constexpr int ST_WBUF = ST_WPENT + ST_WDYENT;    // entries per buffer
constexpr int ST_NCOL = 392, ST_NT = 25;         // dW columns, 16-column tiles

static int g_conv_stem_v = 1;
TAM_KNOB(g_conv_stem_v)
static int g_conv_stem_ref() { return g_conv_stem_v; }

struct StemWArgs {
  const bf16_t* dy;     // [N][P][Q][64]
  const bf16_t* x;      // [N][H][W][8]
  float* slab;          // [grid][64][392]
  int N, H, W, P, Q, rblocks;
};

__device__ __forceinline__ s16x8_t st_tr_frag(const char* lo, const char* hi) {
  const s16x4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)lo);
  const s16x4_t b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)hi);
  s16x8_t r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

__global__ void __launch_bounds__(512, 1) conv_stem_wgrad_kernel(StemWArgs a) {
  __shared__ __attribute__((aligned(1024))) uint4 buf2[2][ST_WBUF];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int pw = a.W + 6, nent = ST_WPROWS * pw, npch = (nent + 63) / 64;
  const int ngroups = a.N * a.rblocks;
  auto stage = [&](int g, int b) {
    const int n = g / a.rblocks, p0 = (g - n * a.rblocks) * ST_WROWS, h0 = 2 * p0 - 3;
    for (int ch = wv; ch < npch + ST_WDYENT / 64; ch += 8) {
      const void* src = (const void*)g_st_zero;
      if (ch < npch) {                              // patch chunk
        const int i = ch * 64 + lane;
        const int r = i / pw, c = i - r * pw;
        const int h = h0 + r, wc = c - 3;
        if (i < nent && (unsigned)h < (unsigned)a.H && (unsigned)wc < (unsigned)a.W)
          src = (const void*)(a.x + (((long)n * a.H + h) * a.W + wc) * 8);
        __builtin_amdgcn_global_load_lds(src, (st_lds_void_t*)(&buf2[b][ch * 64]), 16, 0, 0);
      } else {                                      // dY chunk: [row][128 px][8 x 16 B]
        const int i = (ch - npch) * 64 + lane;
        const int rr = i >> 10, px = (i >> 3) & 127, part = i & 7;
        if (px < a.Q && p0 + rr < a.P)
          src = (const void*)(a.dy + (((long)n * a.P + p0 + rr) * a.Q + px) * 64 + part * 8);
        __builtin_amdgcn_global_load_lds(src, (st_lds_void_t*)(&buf2[b][ST_WPENT + (ch - npch) * 64]), 16, 0, 0);
      }
    }
  };
  if ((int)blockIdx.x < ngroups) stage(blockIdx.x, 0);

  // wave w: N-tiles w, w + 8, w + 16 (and 24 for wave 0) x all 4 M-tiles
  const int nj = wv == 0 ? 4 : 3;
  const int g16 = lane >> 4, t = lane & 15, q4 = t >> 2, p4 = t & 3;
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // per N-tile: this lane's tap (columns 4 p4 .. +3 of tile j) and channel half
  int toff[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    int tap = 2 * (wv + 8 * jj) + (p4 >> 1);
    tap = tap < 49 ? tap : 48;                      // columns >= 392 are never stored
    const int r = tap / 7, s = tap - 7 * (tap / 7);
    toff[jj] = (r * pw + s) * 16 + (p4 & 1) * 8;    // bytes, relative to (2 pr, 2 q)
  }
  int it = 0;
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x, ++it) {
    const int b = it & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (g + (int)gridDim.x < ngroups) stage(g + gridDim.x, b ^ 1);
    const char* pat = (const char*)&buf2[b][0];
    const char* dyt = (const char*)&buf2[b][ST_WPENT];
    const int n = g / a.rblocks, p0 = (g - n * a.rblocks) * ST_WROWS;
    const int rows = min(ST_WROWS, a.P - p0);
    for (int kstep = 0; kstep < rows * 4; ++kstep) {
      const int pr = kstep >> 2, qb = (kstep & 3) * 32;
      if (qb >= a.Q) continue;
      // this lane's two rows: pixels qb + 8 g16 + q4 (+ 4)
      const int px0 = qb + 8 * g16 + q4, px1 = px0 + 4;
      s16x8_t af[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int cb = (mt * 16 + 4 * p4) * 2;
        af[mt] = st_tr_frag(dyt + ((pr * 128 + px0) * 64) * 2 + cb, dyt + ((pr * 128 + px1) * 64) * 2 + cb);
      }
      const int qa = px0 < a.Q ? px0 : a.Q - 1, qc = px1 < a.Q ? px1 : a.Q - 1;   // dY is zero there
      const char* b0 = pat + ((2 * pr) * pw + 2 * qa) * 16;
      const char* b1 = pat + ((2 * pr) * pw + 2 * qc) * 16;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        if (jj < nj) {
          const s16x8_t bf = st_tr_frag(b0 + toff[jj], b1 + toff[jj]);
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
            acc[mt][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[mt]),
                                                                  __builtin_bit_cast(bf16x8_t, bf), acc[mt][jj], 0, 0,
                                                                  0);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // C[row = 16 mt + 4 g16 + r][col = 16 j + t] -> slab
  float* sl = a.slab + (long)blockIdx.x * 64 * ST_NCOL;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int col = 16 * (wv + 8 * jj) + t;
    if (jj >= nj || col >= ST_NCOL) continue;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) sl[(long)(16 * mt + 4 * g16 + r) * ST_NCOL + col] = acc[mt][jj][r];
  }
}

static int st_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  return cus;
}

static bool stem_geom_ok(const ConvGeom& g) {
  return g.C == 8 && g.K == 64 && g.R == 7 && g.S == 7 && g.stride == 2 && g.pad == 3 && g.dil == 1 &&
         g.W <= ST_PW_MAX - 6 && g.W >= 4 && g.H >= 4 && g.P == (g.H - 1) / 2 + 1 && g.Q == (g.W - 1) / 2 + 1 &&
         g.Q <= 128 && (long)g.N * g.H * g.W * 8 < (1L << 31) && (long)g.N * g.P * g.Q * 64 < (1L << 31);
}

static int stem_wgrad_grid(const ConvGeom& g) {
  const int groups = g.N * ((g.P + ST_WROWS - 1) / ST_WROWS);
  return groups < st_cus() ? groups : st_cus();
}

long conv_stem_wgrad_ws(const ConvGeom& g) {
  if (!g_conv_stem_ref() || !stem_geom_ok(g)) return 0;
  return (long)stem_wgrad_grid(g) * 64 * ST_NCOL;
}

// dw [64][7][7][8] fp32 = (mode ? dw : 0) + stem wgrad; false: not its shape
// (or no scratch: ws must hold conv_stem_wgrad_ws(g) floats)
bool conv_stem_wgrad(const bf16_t* dy, const bf16_t* x, const ConvGeom& g, float* dw, int mode, float* ws,
                     long ws_floats, hipStream_t s) {
  const long need = conv_stem_wgrad_ws(g);
  if (need == 0 || ws == nullptr || ws_floats < need) return false;
  const int grid = stem_wgrad_grid(g);
  StemWArgs a{dy, x, ws, g.N, g.H, g.W, g.P, g.Q, (g.P + ST_WROWS - 1) / ST_WROWS};
  hipLaunchKernelGGL(conv_stem_wgrad_kernel, dim3(grid), dim3(512), 0, s, a);
  wgrad_slab_reduce(ws, grid, 64L * ST_NCOL, dw, mode, s);
  return true;
}

void conv_stem_policy(int p) { g_conv_stem_v = p; }

// y = conv(x, w) (+ bias, ReLU) for the 7x7 / s2 / p3 / 8 -> 64 stem; false
// when the geometry or epilogue is not this kernel's
bool conv_stem_fwd(const bf16_t* x, const bf16_t* w, const ConvGeom& g, const Epi& ep, hipStream_t s) {
  if (!g_conv_stem_v || g.C != 8 || g.K != 64 || g.R != 7 || g.S != 7 || g.stride != 2 || g.pad != 3 ||
      g.dil != 1 || g.W > ST_PW_MAX - 6 || g.W < 4 || g.H < 4)
    return false;
  if (ep.c_f32 || ep.mode != 0 || ep.mask || ep.ldc != 64 || ep.alpha != 1.f || ep.bnx)
    return false;
  if (g.P != (g.H - 1) / 2 + 1 || g.Q != (g.W - 1) / 2 + 1) return false;
  if ((long)g.N * g.H * g.W * 8 >= (1L << 31) || (long)g.N * g.P * g.Q * 64 >= (1L << 31)) return false;
  StemArgs a{x, w, (bf16_t*)ep.c, ep.bias, ep.stats, g.N, g.H, g.W, g.P, g.Q, ep.relu,
             (g.P + ST_ROWS - 1) / ST_ROWS};
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  const int groups = g.N * a.rblocks;
  hipLaunchKernelGGL(conv_stem_fwd_kernel, dim3(groups < cus ? groups : cus), dim3(512), 0, s, a);
  return true;
}

}  // namespace tam
