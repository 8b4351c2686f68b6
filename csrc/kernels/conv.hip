// tiresias_amd — NHWC convolution passes as MFMA implicit GEMMs.
//   fwd  : Y[n,p,q,k]  = sum_{r,s,c} X[n,h(p,r),w(q,s),c] W[k,r,s,c]
//          M = N*P*Q, N_gemm = K, Kdim = R*S*C    (A gathered from X)
//   dgrad: dX[n,h,w,c] = sum_{r,s,k} dY[n,p,q,k] W[k,r,s,c]
//          M = N*H*W, N_gemm = C, Kdim = R*S*K    (A gathered from dY, stride-
//          aware zero taps; B = W^T laid out [C][R][S][K], K-major)
//   wgrad: dW[k,r,s,c] = sum_{n,p,q} dY[n,p,q,k] X[n,h,w,c]
//          M = K, N_gemm = R*S*C, Kdim = N*P*Q    (both operands MN-major,
//          split-K over output pixels with fp32 atomics)
// 1x1 / stride-1 / pad-0 convolutions go straight to the dense GEMM.
#include <cstdlib>

#include "tam/launch.h"
#include "tam/tiles.h"
#include "tam/conv_dma.h"
#include "tam/kernels.h"

namespace tam {

// 1 (default): fwd / stride-1 dgrad with C % 64 == 0 go to the LDS-DMA core
// (conv_dma.h) when the grid fills the chip; 2: LDS-DMA core wherever the
// shape is eligible (tests); 3: as 2 with the 128-row tile variant (tests);
// 0: register-staged igemm only (A/B measurements)
static int g_conv_dma = 1;
TAM_KNOB(g_conv_dma)
void conv_dma_policy(int p) { g_conv_dma = p; }
// split-K of under-filled LDS-DMA conv passes (cd_split_plan): 1 on, 0 off (A/B)
static int g_conv_split = 1;
TAM_KNOB(g_conv_split)
void conv_split_policy(int p) { g_conv_split = p; }
// 64-channel 3x3 stride-1 passes on the halo-tile kernel (conv_dma.h); 0 for
// A/B runs against the tap-gather cores
static int g_conv_halo = [] {
  const char* e = getenv("TAM_CONV_HALO");
  return e ? atoi(e) : 1;
}();
TAM_KNOB(g_conv_halo)
void conv_halo_policy(int p) { g_conv_halo = p; }
static ::tam::KnobReg g_wgrad_force_knobs_[4] = {{"g_wgrad_force0", &g_wgrad_force[0]}, {"g_wgrad_force1", &g_wgrad_force[1]},
                                                  {"g_wgrad_force2", &g_wgrad_force[2]}, {"g_wgrad_force3", &g_wgrad_force[3]}};
void conv_wgrad_force(int bm, int bn, int splits, int noatomic) {
  g_wgrad_force[0] = bm; g_wgrad_force[1] = bn; g_wgrad_force[2] = splits; g_wgrad_force[3] = noatomic;
}

template <int BM, int BN>
static void fwd_tile(const bf16_t* x, const bf16_t* w, const ConvGeom& g, const Epi& ep, int sp,
                     hipStream_t s) {
  const int M = g.N * g.P * g.Q, Kd = g.R * g.S * g.C;
  LdConvFwdA<BM> la{x, g, M, Kd};
  la.with_divs();
  LdKMajor<BN> lb{w, Kd, g.K, Kd};
  launch_igemm<BM, BN>(la, lb, M, g.K, Kd, ep, sp, s);
}

static bool is_pointwise(const ConvGeom& g) {
  return g.R == 1 && g.S == 1 && g.stride == 1 && g.pad == 0;
}

// returns 1 when the path taken accumulated the BN statistics into ep.stats
// (0: none; the BN then reduces the output itself)
// split-K scratch (floats) conv_fwd / conv_dgrad would use on the LDS-DMA
// core for this geometry (0: the pass runs unsplit); the caller allocates it
long conv_fwd_split_ws(const ConvGeom& g) {
  if (!g_conv_dma || g.dil != 1 || !g_conv_split) return 0;
  return conv_dma_split_ws(cd_fwd_args(nullptr, nullptr, g), g_conv_dma >= 2 ? g_conv_dma - 1 : 0);
}
long conv_dgrad_split_ws(const ConvGeom& g) {
  if (!g_conv_dma || g.dil != 1 || g.stride != 1 || !g_conv_split) return 0;
  CDArgs a = cd_dgrad_args(nullptr, nullptr, g, 0, 0);
  const int force = g_conv_dma >= 2 ? g_conv_dma - 1 : (g.C == 64 && a.M >= (1L << 20) ? 1 : 0);
  return conv_dma_split_ws(a, force);
}

// (forcing shallow pointwise convs with BN statistics onto the LDS-DMA core,
// or accumulating their statistics in the igemm epilogue, measured neutral
// or slower on ResNet-50 -- 9.096 / 9.099 vs 9.084 / 9.095 ms -- and the
// switches were removed in round 6: the cost model decides, and the igemm
// fallback gets a separate bn_stats pass)

int conv_fwd(const bf16_t* x, const bf16_t* w, const ConvGeom& g, Epi ep, hipStream_t s, float* ws,
             long ws_floats) {
  const int M = g.N * g.P * g.Q, Kd = g.R * g.S * g.C;
  if (conv_stem_fwd(x, w, g, ep, s)) return ep.stats ? 1 : 0;   // 7x7/s2 8->64 stem (conv_stem.hip)
  // pointwise convs over many pixels (ResNet-50's 56x56 bottleneck 1x1s):
  // the memory-bound short-K kernel, BN statistics in its epilogue
  if (is_pointwise(g) && !ep.c_f32 && ep.mode == 0 && !ep.bias && !ep.mask && ep.alpha == 1.f &&
      gemm_pw(x, g.C, w, g.C, (bf16_t*)ep.c, ep.ldc, M, g.K, g.C, nullptr, 0, ep.stats, ep.relu, s))
    return ep.stats ? 1 : 0;
  if (g_conv_dma && g.dil == 1) {
    CDArgs a = cd_fwd_args(x, w, g);
    if (g_conv_halo && launch_conv_halo(a, ep, s)) return ep.stats ? 1 : 0;
    const int force = g_conv_dma >= 2 ? g_conv_dma - 1 : 0;
    const int bm = launch_conv_dma(a, ep, s, force, ws, ws_floats);
    if (bm) return ep.stats ? 1 : 0;
  }
  if (is_pointwise(g)) {
    ep.stats = nullptr;
    gemm(x, g.C, true, w, g.C, true, M, g.K, g.C, ep, false, s);
    return 0;
  }
  ep.stats = nullptr;
  TileChoice t = choose_tiles(M, g.K, Kd, false);
  switch (t.cfg) {
    case 0: fwd_tile<128, 128>(x, w, g, ep, 1, s); break;
    case 1: fwd_tile<128, 64>(x, w, g, ep, 1, s); break;
    case 2: fwd_tile<64, 128>(x, w, g, ep, 1, s); break;
    default: fwd_tile<64, 64>(x, w, g, ep, 1, s); break;
  }
  return 0;
}

template <int BM, int BN>
static void dgrad_tile(const bf16_t* dy, const bf16_t* wt, const ConvGeom& g, const Epi& ep,
                       hipStream_t s) {
  const int M = g.N * g.H * g.W, Kd = g.R * g.S * g.K;
  LdConvDgradA<BM> la{dy, g, M, Kd};
  la.with_divs();
  LdKMajor<BN> lb{wt, Kd, g.C, Kd};
  launch_igemm<BM, BN>(la, lb, M, g.C, Kd, ep, 1, s);
}

// returns 1 when the BN-backward sums (Epi::bnx) were accumulated into
// ep.stats -- only the single-launch stride-1 LDS-DMA path produces them;
// every other path clears ep.stats and returns 0
int conv_dgrad(const bf16_t* dy, const bf16_t* w, const bf16_t* wt, const ConvGeom& g, Epi ep,
               hipStream_t s, float* ws, long ws_floats) {
  const int M = g.N * g.H * g.W, Kd = g.R * g.S * g.K;
  if (wt && g_conv_dma && g.dil == 1 && g.stride == 1) {
    // rows = dX pixels over an H x W grid, gathered from dY (P x Q x K), B = Wt [C][R][S][K]
    CDArgs a = cd_dgrad_args(dy, wt, g, 0, 0);
    if (g_conv_halo && launch_conv_halo(a, ep, s)) return ep.stats ? 1 : 0;
    // 64-channel dX over >= 1M pixels (VGG-16's 224x224 layer): the 64-wide
    // DMA tile beats the igemm although Kd < 1024 (measured 422 -> 364 us);
    // the cost model's 64-column rule is tuned for ResNet's shallower grids
    static const long dg64_min_m = [] {
      const char* e = getenv("TAM_DGRAD64_MIN_M");     // A/B of the 64-channel rule
      return e ? atol(e) : (1L << 20);
    }();
    const int force = g_conv_dma >= 2 ? g_conv_dma - 1 : (g.C == 64 && a.M >= dg64_min_m ? 1 : 0);
    const int bm = launch_conv_dma(a, ep, s, force, ws, ws_floats);
    if (bm) return ep.stats ? 1 : 0;
  }
  ep.stats = nullptr;
  ep.bnx = nullptr;
  if (wt && g_conv_dma && g.dil == 1 && g.stride > 1 && g.K % 64 == 0 && g.C % 64 == 0 &&
      ep.mode == 0 && !ep.c_f32 && g.stride * g.stride <= 4) {
    // strided dgrad = one stride-1 sub-convolution per output parity class
    // (dX pixels with h % s == ph get only the taps r == ph + pad (mod s));
    // classes without taps (1x1 stride 2: 3 of 4) are zero
    CDArgs cls[4];
    bool ok = true, empty = false;
    for (int ph = 0, i = 0; ph < g.stride; ++ph)
      for (int pw = 0; pw < g.stride; ++pw, ++i) {
        cls[i] = cd_dgrad_args(dy, wt, g, ph, pw);
        if (cls[i].ntaps == 0) empty = true;
        else ok = ok && conv_dma_pick_bn(cls[i].M, cls[i].Ng, cls[i].Kd, 1) != 0;
      }
    if (ok) {
      if (empty) zero_async(ep.c, (size_t)M * g.C * sizeof(bf16_t), s);
      // every non-empty class in ONE launch (policy 3, tests: one launch per
      // class on the 128-row tile)
      CDArgs live[4];
      int n = 0;
      for (int i = 0; i < g.stride * g.stride; ++i)
        if (cls[i].ntaps) live[n++] = cls[i];
      if (g_conv_dma == 3 || !launch_conv_dma_multi(live, n, ep, s))
        for (int i = 0; i < n; ++i) launch_conv_dma(live[i], ep, s, g_conv_dma == 3 ? 2 : 1);
      return 0;
    }
  }
  if (is_pointwise(g)) {
    // many pixels: the short-K kernel on the re-laid Wt [C][K] (K-major B),
    // ReLU-backward mask in its epilogue
    if (wt && !ep.c_f32 && ep.mode == 0 && !ep.bias && ep.alpha == 1.f && !ep.relu &&
        gemm_pw(dy, g.K, wt, g.K, (bf16_t*)ep.c, ep.ldc, M, g.C, g.K, ep.mask, ep.ldm, nullptr, 0, s))
      return 0;
    // dX[m][c] = sum_k dY[m][k] W[k][c]  -> B(k,n) = W[k*C + c], MN-major
    gemm(dy, g.K, true, w, g.C, false, M, g.C, g.K, ep, false, s);
    return 0;
  }
  TileChoice t = choose_tiles(M, g.C, Kd, false);
  switch (t.cfg) {
    case 0: dgrad_tile<128, 128>(dy, wt, g, ep, s); break;
    case 1: dgrad_tile<128, 64>(dy, wt, g, ep, s); break;
    case 2: dgrad_tile<64, 128>(dy, wt, g, ep, s); break;
    default: dgrad_tile<64, 64>(dy, wt, g, ep, s); break;
  }
  return 0;
}

template <int BM, int BN>
static void wgrad_tile(const bf16_t* dy, const bf16_t* x, const ConvGeom& g, const Epi& ep, int sp,
                       hipStream_t s) {
  const int Mred = g.N * g.P * g.Q, Nc = g.R * g.S * g.C;
  LdMNMajor<BM> la{dy, g.K, g.K, Mred};
  LdConvWgradB<BN> lb{x, g, Mred, Nc};
  lb.with_divs();
  launch_igemm<BM, BN>(la, lb, g.K, Nc, Mred, ep, sp, s);
}

// 64-channel 3x3 stride-1 weight gradients on the patch-staged kernel
// (conv_dma.h conv_wgrad_c64_kernel): 1 (default) on wherever the caller's
// stream does not run beside the main stream (conv_wgrad allow_patch), 0
// off, >= 2: forced with that many blocks per 64-channel k-slice (tests,
// grid sweeps). VGG-16 (tools/ab_vgg_c64.py): eager gang path without the
// weight-gradient side stream 7.71 -> 7.41 ms; hipGraph with the side stream
// unchanged (the kernel's 120 KB of LDS per CU starves co-running kernels
// there, so it is routed around: 7.42 -> 7.52 ms when it was not)
static int g_wgrad_c64 = 1;
TAM_KNOB(g_wgrad_c64) TAM_KNOB(g_wgrad_slab)
void conv_wgrad_c64_policy(int p) { g_wgrad_c64 = p; }
void conv_wgrad_order(int flat) { g_wgrad_flat = flat; }
void conv_wgrad_slab_policy(int p) { g_wgrad_slab = p; }
long conv_wgrad_split_ws(const ConvGeom& g) {
  const long stem = conv_stem_wgrad_ws(g);     // the stem kernel's per-CU partial slabs
  if (stem > 0) return stem;
  if (!g_conv_dma || (is_pointwise(g) && (long)g.N * g.P * g.Q < 100352 && g_conv_dma < 2)) return 0;
  return wgrad_dma_slab_floats(g, g_conv_dma >= 2);
}

// dbias (optional, fp32 [K]): += the bias gradient sum_m dY[m][k], fused
// into whichever wgrad kernel runs (each reads dY anyway); returns 1 when
// fused, 0 when the caller must add it itself (the LDS-DMA GEMM route of a
// pointwise wgrad has no such epilogue)
// allow_patch: the caller's stream does not run beside the main compute
// stream (the patch kernel holds 120 KB of LDS per CU for its whole run and
// starves co-running kernels: VGG-16's graph step with the weight gradients
// on the side stream measured 7.42 -> 7.52 ms with it)
int conv_wgrad(const bf16_t* dy, const bf16_t* x, const ConvGeom& g, Epi ep, hipStream_t s, float* dbias,
               bool allow_patch, float* ws, long ws_floats, int* slab_defer) {
  if (slab_defer) *slab_defer = 0;
  const int Mred = g.N * g.P * g.Q, Nc = g.R * g.S * g.C;
  if (!dbias && ep.c_f32 && ep.ldc == Nc && ep.mode <= 1 &&
      conv_stem_wgrad(dy, x, g, (float*)ep.c, ep.mode, ws, ws_floats, s))   // 7x7/s2 8->64 stem
    return 0;
  // the patch kernel only for 64 -> 64 (VGG-16's 224x224 layer: 313 vs 343 us
  // on the DMA kernel); 64 -> 128 at 112x112 runs 172 us on it vs 136 us on
  // the DMA kernel's streaming tiles (profiles/r4/wgrad_sweep_vgg224.json)
  if (g_conv_dma && g_wgrad_c64 && (allow_patch || g_wgrad_c64 >= 2) && (g.K == 64 || g_wgrad_c64 >= 2) &&
      ep.c_f32 && ep.ldc == Nc && ep.mode <= 1 &&
      launch_conv_wgrad_c64(dy, x, (float*)ep.c, g, ep.mode, g_wgrad_c64 >= 2 ? g_wgrad_c64 : 0, s,
                            g_conv_dma >= 2 || g_wgrad_c64 >= 2, dbias))
    return dbias ? 1 : 0;
  // pointwise wgrads with a short pixel reduction (ResNet-50 stages 2-4,
  // <= 28x28 at batch 64) are plain dY^T X GEMMs that the routed GEMM runs
  // faster (14x14 256->1024: 24.0 vs 30.7 us, 7x7 512->2048: 22.9 vs 29.5;
  // tools/sweep_wgrad.py, profiles/r4/wgrad_sweep_*.json); the 56x56 ones
  // stay on the DMA kernel (19.6 vs 57 us at 64->64)
  const bool pw_gemm = is_pointwise(g) && Mred < 100352 && g_conv_dma < 2;
  if (g_conv_dma && !pw_gemm && ep.c_f32 && ep.ldc == Nc && ep.mode <= 1 &&
      launch_conv_wgrad_dma(dy, x, (float*)ep.c, g, ep.mode, s, g_conv_dma >= 2, dbias, ws, ws_floats,
                            slab_defer))
    return dbias ? 1 : 0;
  if (is_pointwise(g)) {
    // dW[k][c] = sum_m dY[m][k] X[m][c]: A(k', m) = dY[m*K + k'], B(m, c) = X[m*C + c]
    const bool big = gemm_select_big_p8(false, false, g.K, g.C, Mred, g.K, g.C);
    if (!big) ep.colsum_a = dbias;
    gemm(dy, g.K, false, x, g.C, false, g.K, g.C, Mred, ep, true, s);
    return (dbias && !big) ? 1 : 0;
  }
  ep.colsum_a = dbias;                    // the gather igemm: A = dY, M-major
  TileChoice t = choose_tiles(g.K, Nc, Mred, true);
  if (t.splits > 1 && Nc >= 256) {       // (stem-like Nc = 72 stays on 64x64 tiles)
    // split-K regime (tiny dW, huge pixel reduction): every N tile re-reads
    // all of dY, so prefer the widest tile and let split-K fill the CUs
    // (C=64 3x3 wgrads: 9 -> 5 passes over dY)
    const int cfg = g.K > 64 ? 0 : 2;
    const long tiles = (long)cdiv(g.K, cfg == 0 ? 128 : 64) * cdiv(Nc, 128);
    const int ktiles = cdiv(Mred, IG_BK);
    int sp = (int)((512 + tiles - 1) / tiles);
    if (sp > ktiles / 4) sp = ktiles / 4;
    if (sp > 256) sp = 256;
    t = TileChoice{cfg, sp < 1 ? 1 : sp};
  }
  prepare_split(ep, t.splits, g.K, Nc, s);
  switch (t.cfg) {
    case 0: wgrad_tile<128, 128>(dy, x, g, ep, t.splits, s); break;
    case 1: wgrad_tile<128, 64>(dy, x, g, ep, t.splits, s); break;
    case 2: wgrad_tile<64, 128>(dy, x, g, ep, t.splits, s); break;
    default: wgrad_tile<64, 64>(dy, x, g, ep, t.splits, s); break;
  }
  return dbias ? 1 : 0;
}

void wgrad_slab_reduce_many(const float* const* ws, const int* sp, const long* mn, float* const* dw,
                            const int* mode, int n, hipStream_t s) {
  wgrad_slab_reduce_batch(ws, sp, mn, dw, mode, n, s);
}

// wt[c][(r*S+s)*K + k] = w[k][(r*S+s)*C + c]
__global__ void conv_weight_t_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wt, int K,
                                     int RS, int C) {
  const long total = (long)K * RS * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int k = (int)(i % K);
    const long t = i / K;
    const int rs = (int)(t % RS);
    const int c = (int)(t / RS);
    wt[i] = w[((long)k * RS + rs) * C + c];
  }
}

// Every conv weight of a model re-laid [K][RS][C] -> [C][RS][K] in ONE launch
// (the dgrad B operand), 64 x 64 (k, c) tiles through LDS so both the read
// (along c) and the write (along k) are 128-B coalesced rows. Called once per
// training step after the optimizer's weights are final (model forward).
__global__ void __launch_bounds__(256) conv_wt_batch_kernel(WTBatch b) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[64][72];
  int e = 0;
  while (e + 1 < b.n && (int)blockIdx.x >= b.e[e + 1].tile0) ++e;
  const WTEntry& en = b.e[e];
  const int tk = (en.K + 63) / 64, tc = (en.C + 63) / 64;
  const int local = blockIdx.x - en.tile0;
  const int rs = local / (tk * tc), r2 = local % (tk * tc);
  const int k0 = (r2 / tc) * 64, c0 = (r2 % tc) * 64;
  if ((en.K & 7) == 0 && (en.C & 7) == 0) {
    // 16-B vectors both ways: rows of 8 c read, 8 k gathered from an LDS
    // column and written as one 16-B chunk (144-B LDS rows: the column
    // gathers of 16 lanes hit 16 different banks)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = threadIdx.x + 256 * u, kk = i >> 3, cv = (i & 7) * 8, k = k0 + kk, c = c0 + cv;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (k < en.K && c < en.C) v = *(const uint4*)(en.w + ((long)k * en.RS + rs) * en.C + c);
      *(uint4*)&tile[kk][cv] = v;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = threadIdx.x + 256 * u, cc = i >> 3, kv = (i & 7) * 8, k = k0 + kv, c = c0 + cc;
      if (k >= en.K || c >= en.C) continue;
      uint32_t w4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        w4[q] = (uint32_t)tile[kv + 2 * q][cc] | ((uint32_t)tile[kv + 2 * q + 1][cc] << 16);
      *(uint4*)(en.wt + ((long)c * en.RS + rs) * en.K + k) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
    return;
  }
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int kk = i >> 6, cc = i & 63, k = k0 + kk, c = c0 + cc;
    tile[kk][cc] = (k < en.K && c < en.C) ? en.w[((long)k * en.RS + rs) * en.C + c] : (bf16_t)0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int cc = i >> 6, kk = i & 63, k = k0 + kk, c = c0 + cc;
    if (k < en.K && c < en.C) en.wt[((long)c * en.RS + rs) * en.K + k] = tile[kk][cc];
  }
}

void conv_weight_t_batch(WTBatch& b, hipStream_t s) {
  int tiles = 0;
  for (int i = 0; i < b.n; ++i) {
    b.e[i].tile0 = tiles;
    tiles += b.e[i].RS * ((b.e[i].K + 63) / 64) * ((b.e[i].C + 63) / 64);
  }
  if (tiles > 0) hipLaunchKernelGGL(conv_wt_batch_kernel, dim3(tiles), dim3(256), 0, s, b);
}

void conv_weight_t(const bf16_t* w, bf16_t* wt, const ConvGeom& g, hipStream_t s) {
  const long total = (long)g.K * g.R * g.S * g.C;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(conv_weight_t_kernel, dim3(blocks), dim3(256), 0, s, w, wt, g.K, g.R * g.S,
                     g.C);
}

}  // namespace tam
