// tiresias_amd — fused LSTM cell pointwise (GNMT). The gate pre-activations
// G = X W_ih^T + h W_hh^T + b are produced by the MFMA GEMM (fp32 output,
// the x-part for all timesteps in one GEMM, the h-part accumulated per step);
// this kernel does every elementwise op of the cell in one pass and caches the
// activations the backward needs. Gate order: i, f, g, o.
#include "tam/common.h"
#include "tam/kernels.h"

#include <map>
#include <mutex>

namespace tam {

__device__ __forceinline__ float tanhf_(float x) { return 1.f - 2.f / (__expf(2.f * x) + 1.f); }

__global__ void lstm_fwd_kernel(const float* __restrict__ G, const float* __restrict__ cp,
                                float* __restrict__ c, bf16_t* __restrict__ hb,
                                float* __restrict__ hf, float* __restrict__ act, int B, int Hd) {
  const long n = (long)B * Hd;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < n;
       idx += (long)gridDim.x * blockDim.x) {
    const int b = (int)(idx / Hd), j = (int)(idx % Hd);
    const float* g = G + (long)b * 4 * Hd;
    const float i_ = sigmoidf_(g[j]), f_ = sigmoidf_(g[Hd + j]);
    const float g_ = tanhf_(g[2 * Hd + j]), o_ = sigmoidf_(g[3 * Hd + j]);
    const float cn = f_ * (cp ? cp[idx] : 0.f) + i_ * g_;
    const float tc = tanhf_(cn);
    const float h = o_ * tc;
    c[idx] = cn;
    if (hb) hb[idx] = f2bf(h);
    if (hf) hf[idx] = h;
    float* a = act + (long)b * 5 * Hd;
    a[j] = i_; a[Hd + j] = f_; a[2 * Hd + j] = g_; a[3 * Hd + j] = o_; a[4 * Hd + j] = tc;
  }
}

__global__ void lstm_bwd_kernel(const float* __restrict__ act, const float* __restrict__ cp,
                                const float* __restrict__ dh, const float* __restrict__ dcn,
                                float* __restrict__ dG, float* __restrict__ dcp,
                                bf16_t* __restrict__ dGb, int B, int Hd) {
  const long n = (long)B * Hd;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < n;
       idx += (long)gridDim.x * blockDim.x) {
    const int b = (int)(idx / Hd), j = (int)(idx % Hd);
    const float* a = act + (long)b * 5 * Hd;
    const float i_ = a[j], f_ = a[Hd + j], g_ = a[2 * Hd + j], o_ = a[3 * Hd + j], tc = a[4 * Hd + j];
    const float dhv = dh ? dh[idx] : 0.f;
    const float dc = dhv * o_ * (1.f - tc * tc) + (dcn ? dcn[idx] : 0.f);
    const float cpv = cp ? cp[idx] : 0.f;
    const float di = dc * g_ * i_ * (1.f - i_);
    const float df = dc * cpv * f_ * (1.f - f_);
    const float dg = dc * i_ * (1.f - g_ * g_);
    const float dO = dhv * tc * o_ * (1.f - o_);
    const long gb = (long)b * 4 * Hd;
    if (dG) { dG[gb + j] = di; dG[gb + Hd + j] = df; dG[gb + 2 * Hd + j] = dg; dG[gb + 3 * Hd + j] = dO; }
    if (dGb) {
      dGb[gb + j] = f2bf(di); dGb[gb + Hd + j] = f2bf(df);
      dGb[gb + 2 * Hd + j] = f2bf(dg); dGb[gb + 3 * Hd + j] = f2bf(dO);
    }
    if (dcp) dcp[idx] = dc * f_;
  }
}

// ---------------------------------------------------------------------------
// Fused forward timestep: gates = Gx[t] + h_{t-1} W_hh^T, then the cell.
// One launch per timestep instead of {split-K GEMM with atomics, cell kernel}.
// Workgroup = 4 hidden units (j0..j0+3) = 16 gate rows ordered
// n = gate*4 + unit, so the cells of those units are local to the WG:
// Hd/4 workgroups (256 for GNMT's 1024) -> one per CU, no atomics.
// The step is latency-bound (h_{t-1} comes from the previous launch), so the
// WG is sized for ONE memory round trip: waves = MT batch tiles x KS K-slices,
// each wave issues all 8 k-steps (32 x 8 = 256 of K) of h / W_hh fragment
// loads (16 B per lane per operand) at once, 8 MFMAs, partial 16x16 tile to
// LDS; the cell operands (Gx, c_{t-1}) are prefetched before the MFMAs.
constexpr int LS_K = 8;   // k-steps (of 32) per wave

template <int KS>
__global__ void __launch_bounds__(1024) lstm_step_fwd_kernel(
    const float* __restrict__ gx, const bf16_t* __restrict__ w, const bf16_t* __restrict__ hp,
    const float* __restrict__ cp, float* __restrict__ c, bf16_t* __restrict__ hb,
    float* __restrict__ act, int B, int Hd, int MT) {
  __shared__ float part[16][16][17];   // [wave][batch row][gate row]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int mt = wv / KS, ks = wv % KS;
  const int j0 = blockIdx.x * 4;
  const int n = lane & 15;
  const bf16_t* wrow = w + ((long)(n >> 2) * Hd + j0 + (n & 3)) * Hd;
  for (int m0 = 0; m0 < B; m0 += 16 * MT) {
    // prefetch this thread's cell operands (thread t < 64*MT owns one cell)
    const int t = threadIdx.x;
    const bool cell = t < 64 * MT;
    const int cb = m0 + (t >> 2), cu = t & 3;
    float gxv[4] = {0.f, 0.f, 0.f, 0.f}, cpv = 0.f;
    if (cell && cb < B) {
      const float* g = gx + (long)cb * 4 * Hd + j0 + cu;
#pragma unroll
      for (int q = 0; q < 4; ++q) gxv[q] = g[(long)q * Hd];
      if (cp) cpv = cp[(long)cb * Hd + j0 + cu];
    }
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    const int row0 = m0 + 16 * mt;
    if (hp && row0 < B) {
      const bf16_t* hrow = hp + (long)(row0 + (lane & 15)) * Hd;
      for (int kb = ks * 32 * LS_K; kb < Hd; kb += KS * 32 * LS_K) {
        s16x8_t a[LS_K], b[LS_K];
#pragma unroll
        for (int i = 0; i < LS_K; ++i) {
          const int k = kb + 32 * i + 8 * (lane >> 4);
          a[i] = *(const s16x8_t*)(hrow + k);
          b[i] = *(const s16x8_t*)(wrow + k);
        }
#pragma unroll
        for (int i = 0; i < LS_K; ++i)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a[i]),
                                                        __builtin_bit_cast(bf16x8_t, b[i]), acc, 0, 0, 0);
      }
    }
    // C/D map: col = lane & 15 (gate row), row = 4*(lane>>4) + r (batch)
#pragma unroll
    for (int r = 0; r < 4; ++r) part[wv][4 * (lane >> 4) + r][lane & 15] = acc[r];
    __syncthreads();
    if (cell && cb < B) {
      const int bl = t >> 2, mtc = bl >> 4, br = bl & 15;
      float gs[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v = gxv[q];
#pragma unroll
        for (int k = 0; k < KS; ++k) v += part[mtc * KS + k][br][q * 4 + cu];
        gs[q] = v;
      }
      const float i_ = sigmoidf_(gs[0]), f_ = sigmoidf_(gs[1]), g_ = tanhf_(gs[2]), o_ = sigmoidf_(gs[3]);
      const int j = j0 + cu;
      const long idx = (long)cb * Hd + j;
      const float cn = f_ * cpv + i_ * g_;
      const float tc = tanhf_(cn);
      c[idx] = cn;
      hb[idx] = f2bf(o_ * tc);
      float* a = act + (long)cb * 5 * Hd;
      a[j] = i_; a[Hd + j] = f_; a[2 * Hd + j] = g_; a[3 * Hd + j] = o_; a[4 * Hd + j] = tc;
    }
    __syncthreads();
  }
}

void lstm_step_forward(const float* gx, const bf16_t* w_hh, const bf16_t* h_prev, const float* c_prev,
                       float* c_out, bf16_t* h_out, float* act, int B, int Hd, hipStream_t s) {
  // K-slices: largest of 4/2/1 dividing Hd/256; batch tiles so waves <= 16
  const int q = Hd / 256;
  const int KS = q % 4 == 0 ? 4 : (q % 2 == 0 ? 2 : 1);
  int MT = 16 / KS;
  if (MT > B / 16) MT = B / 16;
  const dim3 blk(64 * MT * KS);
  if (KS == 4)
    hipLaunchKernelGGL(lstm_step_fwd_kernel<4>, dim3(Hd / 4), blk, 0, s, gx, w_hh, h_prev, c_prev, c_out,
                       h_out, act, B, Hd, MT);
  else if (KS == 2)
    hipLaunchKernelGGL(lstm_step_fwd_kernel<2>, dim3(Hd / 4), blk, 0, s, gx, w_hh, h_prev, c_prev, c_out,
                       h_out, act, B, Hd, MT);
  else
    hipLaunchKernelGGL(lstm_step_fwd_kernel<1>, dim3(Hd / 4), blk, 0, s, gx, w_hh, h_prev, c_prev, c_out,
                       h_out, act, B, Hd, MT);
}

// ---------------------------------------------------------------------------
// Persistent LSTM recurrence: ONE launch per layer-direction per sequence
// (forward and backward), instead of {recurrent GEMM, cell kernel} per
// timestep.
//
// Workgroup (batch tile of 16 rows, unit tile of 16 hidden units) owns the 64
// gate rows {i,f,g,o} x 16 units, so the cell update is local. B/16 x Hd/16
// workgroups (256 for GNMT's B = 64, H = 1024): one per CU. Each of the 8
// waves keeps its K-slice of those W_hh rows in VGPRs for the whole sequence
// (forward: Hd/8 of K, 64 VGPRs at H = 1024) and reads only its 16-row slice
// of h_{t-1} (the batch tile) each step; the cell state stays in a register.
//
// Step hand-off (only workgroups of the SAME batch tile depend on each other,
// so each batch tile has its own arrival counter on a line of its own): the
// tile's new h (forward) / dG (backward) is staged in LDS, written by ONE wave
// as 8-B write-through (sc1) stores, drained (vmcnt 0), then one lane adds to
// the counter (agent atomic). Consumers: one lane polls the counter with
// relaxed sc1 loads + s_sleep, the workgroup joins at a barrier, and EVERY
// load of handed-off bytes is a 16-B sc1 buffer load -- no release / acquire fence
// (guide: Guideline 16 / microarch visibility table, row 1). The spin is
// bounded: a stuck barrier sets the error word and drains instead of hanging.
// Co-residency is checked on the host: the launcher refuses (returns false)
// unless TWO such grids fit at once (two GNMT jobs sharing a GPU).
// ---------------------------------------------------------------------------
constexpr int PL_W = 8;          // waves per workgroup
// poll bound of one hand-off wait: 2^16 relaxed sc1 polls + s_sleep(1) is
// ~50-100 ms, four orders of magnitude above a step's hand-off (~4-6 us)
// even behind another job's kernels; a grid that cannot become co-resident
// (two jobs' different persistent kernels on one GPU) gives up that fast
constexpr unsigned PL_SPIN = 1u << 16;
// Sticky count of persistent-grid barrier timeouts on this device (every job
// of the process): the kernels never hang, but a timed-out step computed on
// h / dG that had not arrived. The host reads it after the round's
// synchronize (lstm_persist_timeouts) and the trainer raises + falls back to
// the per-step path (models/gnmt.py). g_pl_spin is the poll bound (tests
// shrink it to force a timeout).
__device__ unsigned g_pl_timeouts;
__device__ unsigned g_pl_spin = PL_SPIN;
#ifndef PL_BCH
#define PL_BCH 16         // backward: dG fragment loads in flight per chunk
#endif
typedef __attribute__((address_space(1))) unsigned pl_gu32;
typedef __attribute__((address_space(1))) unsigned long long pl_gu64;
#define PL_RLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

// sync layout (int32 words): [0] error flag; [32 * (1 + bt * ns + k)] arrival
// counter k < ns of batch tile bt, each on a 128-B line of its own. With
// ns > 1 the Hd/U producers of a batch tile arrive on ns counters (unit tile
// ut on counter ut % ns): a fan-in of Hd/U atomics on one word serialises at
// ~12 ns each (MI355X_MICROARCH.md, "fanin"); the consumer's first ns lanes
// poll one counter each.
constexpr int PL_NS_MAX = 4;
__device__ __forceinline__ void pl_signal(unsigned* sync, int line) {
  // caller: the ONE storing wave, after its sc1 stores
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add((pl_gu32*)(sync + 32 * (1 + line)), 1u, PL_RLX);
}

// target: arrivals expected on EACH of the ns counters line0 .. line0 + ns - 1
// job_err (nullable): the launching JOB's own timeout word (models/gnmt.py
// GNMT.err[0]), so one job's timeout guards only that job's optimizer step
__device__ __forceinline__ void pl_wait(unsigned* sync, int line0, int ns, unsigned target, unsigned* job_err) {
  if (threadIdx.x < (unsigned)ns) {
    unsigned polls = 0;
    const unsigned spin = g_pl_spin;
    while (__hip_atomic_load((pl_gu32*)(sync + 32 * (1 + line0 + threadIdx.x)), PL_RLX) < target) {
      __builtin_amdgcn_s_sleep(1);
      // a barrier of this launch (or an earlier launch of the same job's
      // step) already timed out: the step's update is skipped anyway, so
      // drain instead of paying the full bound at every later wait
      if ((++polls & 255) == 0 &&
          (__hip_atomic_load((pl_gu32*)sync, PL_RLX) != 0u ||
           (job_err != nullptr && __hip_atomic_load((pl_gu32*)job_err, PL_RLX) != 0u)))
        break;
      if (polls > spin) {
        __hip_atomic_fetch_or((pl_gu32*)sync, 1u, PL_RLX);
        __hip_atomic_fetch_add((pl_gu32*)&g_pl_timeouts, 1u, PL_RLX);
        if (job_err != nullptr) __hip_atomic_fetch_add((pl_gu32*)job_err, 1u, PL_RLX);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps loads below
}

// 16 B of handed-off bf16: one buffer_load_dwordx4 with sc1 (aux 16) through
// a descriptor built from wave-uniform kernel arguments
typedef unsigned int pl_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pl_rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ s16x8_t pl_ld16(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  const pl_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16);
  return __builtin_bit_cast(s16x8_t, v);
}

// CH = unit halves per workgroup: 16 * CH hidden units, 8 * CH waves (8 K-
// slices x CH unit halves). CH = 2 halves the grid (and the per-step h / dG
// traffic, which every workgroup of a batch tile re-reads) at the same bytes
// per workgroup.
template <int KW, int CH>   // KW: k-steps of 32 per wave = Hd / (32 * PL_W)
__global__ void __launch_bounds__(64 * PL_W * CH, 4) lstm_persist_fwd_kernel(
    const float* __restrict__ gx, const bf16_t* __restrict__ w, bf16_t* hs, float* __restrict__ cs,
    float* __restrict__ act, int T, int B, int Hd, int reverse, unsigned* sync, int ns, unsigned* job_err) {
  constexpr int U = 16 * CH;                 // units per workgroup
  __shared__ float red[PL_W][16][4 * U + 1];
  __shared__ __attribute__((aligned(16))) bf16_t hbuf[16][U];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ksl = wv % PL_W, half = wv / PL_W;
  const int nbt = B / 16;
  const int bt = blockIdx.x % nbt, ut = blockIdx.x / nbt;
  const int b0 = bt * 16, j0 = ut * U;
  const int kb = ksl * KW * 32 + 8 * (lane >> 4);
  // W_hh rows {i,f,g,o} x this wave's 16 units, its K-slice, as MFMA B fragments
  s16x8_t wf[4][KW];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int ks = 0; ks < KW; ++ks)
      wf[g][ks] = *(const s16x8_t*)(w + (long)(g * Hd + j0 + 16 * half + (lane & 15)) * Hd + kb + 32 * ks);
  const __amdgpu_buffer_rsrc_t hrs = pl_rsrc(hs, (long)T * B * Hd * 2);
  const bool cell = threadIdx.x < 16 * U;
  const int cr = threadIdx.x / U, cu = threadIdx.x % U;
  float c_reg = 0.f;
  for (int s = 0; s < T; ++s) {
    const int t = reverse ? T - 1 - s : s;
    float gxv[4] = {0.f, 0.f, 0.f, 0.f};
    if (cell) {
      const float* g = gx + ((long)t * B + b0 + cr) * 4 * Hd + j0 + cu;
#pragma unroll
      for (int q = 0; q < 4; ++q) gxv[q] = g[(long)q * Hd];
    }
    f32x4_t acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (s > 0) {
      const int tp = reverse ? t + 1 : t - 1;
      const unsigned hoff = (unsigned)((((long)tp * B + b0 + (lane & 15)) * Hd + kb) * 2);
      s16x8_t ha[KW];
#pragma unroll
      for (int ks = 0; ks < KW; ++ks) ha[ks] = pl_ld16(hrs, hoff + 64 * ks);
#pragma unroll
      for (int ks = 0; ks < KW; ++ks)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, ha[ks]),
                                                           __builtin_bit_cast(bf16x8_t, wf[g][ks]),
                                                           acc[g], 0, 0, 0);
    }
    // C/D map: col = lane & 15 (unit), row = 4*(lane>>4) + r (batch)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[ksl][4 * (lane >> 4) + r][g * U + 16 * half + (lane & 15)] = acc[g][r];
    __syncthreads();
    if (cell) {
      float gs[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v = gxv[q];
#pragma unroll
        for (int k = 0; k < PL_W; ++k) v += red[k][cr][q * U + cu];
        gs[q] = v;
      }
      const float i_ = sigmoidf_(gs[0]), f_ = sigmoidf_(gs[1]), g_ = tanhf_(gs[2]), o_ = sigmoidf_(gs[3]);
      const float cn = f_ * c_reg + i_ * g_;
      const float tc = tanhf_(cn);
      const long row = (long)t * B + b0 + cr;
      const int j = j0 + cu;
      cs[row * Hd + j] = cn;
      hbuf[cr][cu] = f2bf(o_ * tc);
      float* a = act + row * 5 * Hd;
      a[j] = i_; a[Hd + j] = f_; a[2 * Hd + j] = g_; a[3 * Hd + j] = o_; a[4 * Hd + j] = tc;
      c_reg = cn;
    }
    __syncthreads();
    if (wv == 0) {
      // 16 rows x U units of h_t: (64 x CH) x 8 B, write-through
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int idx = u * 64 + lane, r = idx / (4 * CH), q = idx % (4 * CH);
        const unsigned long long v = *(const unsigned long long*)&hbuf[r][4 * q];
        __hip_atomic_store((pl_gu64*)(hs + ((long)t * B + b0 + r) * Hd + j0 + 4 * q), v, PL_RLX);
      }
      if (s + 1 < T) pl_signal(sync, bt * ns + ut % ns);
    }
    if (s + 1 < T) pl_wait(sync, bt * ns, ns, (unsigned)(s + 1) * (unsigned)(Hd / U / ns), job_err);
  }
}

// Backward: dh_t = dH_t + dG_{t+1} W_hh[:, units] (t+1 = the step processed
// after t in the forward order), then the cell backward; dG_t (bf16) is both
// the next step's operand and the weight-gradient GEMMs' input. Each wave
// keeps its K-slice (4Hd/8) of W_hh's 16 columns (its unit half) in VGPRs.
template <int KW, int CH>   // KW: k-steps of 32 per wave = 4 Hd / (32 * PL_W)
__global__ void __launch_bounds__(64 * PL_W * CH, 4) lstm_persist_bwd_kernel(
    const float* __restrict__ act, const float* __restrict__ cs, const float* __restrict__ dH,
    const bf16_t* __restrict__ w, bf16_t* dG, int T, int B, int Hd, int reverse, unsigned* sync, int ns,
    int dh_bf16, int ldh, unsigned* job_err) {
  constexpr int U = 16 * CH;
  // W fragments: the first KWR k-steps in VGPRs, the rest in LDS (the whole
  // slice in VGPRs needs > 128 of them and spills; CH = 1 only: 2 blocks/CU
  // of 8 waves x (KW/2) x 1 KB fit the 160 KB)
  constexpr int KWL = CH == 1 ? KW / 2 : 0, KWR = KW - KWL;
  constexpr int RED_BYTES = PL_W * 16 * (U + 1) * 4, STAGE_BYTES = PL_W * CH * 32 * 16 * 2;
  __shared__ __attribute__((aligned(16))) char misc[RED_BYTES > STAGE_BYTES ? RED_BYTES : STAGE_BYTES];
  __shared__ __attribute__((aligned(16))) s16x8_t wlds[KWL > 0 ? PL_W * CH : 1][KWL > 0 ? KWL : 1][64];
  __shared__ __attribute__((aligned(16))) bf16_t gbuf[16][4 * U];
  auto red = (float(*)[16][U + 1])misc;
  auto wstage = (bf16_t(*)[32][16])misc;     // prologue only, aliases red
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ksl = wv % PL_W, half = wv / PL_W;
  const int nbt = B / 16;
  const int bt = blockIdx.x % nbt, ut = blockIdx.x / nbt;
  const int b0 = bt * 16, j0 = ut * U;
  const int kb = ksl * KW * 32 + 8 * (lane >> 4);
  // B fragment (k, n) = W_hh[k][j0 + 16 half + n]: 8 consecutive k of one
  // column, gathered once through a per-wave LDS slab (32 rows x 16 columns
  // per k-step, 16-B coalesced loads), each lane then picking its 8 k
  s16x8_t wf[KWR];
  {
    const int kw0 = ksl * KW * 32;
    const bf16_t* wcol = w + j0 + 16 * half;
#pragma unroll
    for (int ks = 0; ks < KW; ++ks) {
      const int r = lane >> 1, hh = lane & 1;
      *(uint4*)&wstage[wv][r][8 * hh] = *(const uint4*)(wcol + (long)(kw0 + 32 * ks + r) * Hd + 8 * hh);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      s16x8_t f;
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = (short)wstage[wv][8 * (lane >> 4) + e][lane & 15];
      if (ks < KWR) wf[ks < KWR ? ks : 0] = f;
      else wlds[wv][ks - KWR][lane] = f;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();                           // wstage (aliases red) retired
  const __amdgpu_buffer_rsrc_t grs = pl_rsrc(dG, (long)T * B * 4 * Hd * 2);
  const bool cell = threadIdx.x < 16 * U;
  const int cr = threadIdx.x / U, cu = threadIdx.x % U;
  float dc_reg = 0.f;
  // cell operands of a step (dH, the 5 saved activations, c_{t-1}) do not
  // depend on the recurrence: they are loaded one step AHEAD, issued after
  // the hand-off signal and before the wait, so their HBM latency hides
  // behind the wait + the next MFMA chain instead of following it
  float nx_dh = 0.f, nx_a[5] = {0.f, 0.f, 0.f, 0.f, 0.f}, nx_cp = 0.f;
  auto load_cell = [&](int s) {
    const int t = reverse ? s : T - 1 - s;
    const int fwd_idx = reverse ? T - 1 - t : t;
    const long row = (long)t * B + b0 + cr;
    const int j = j0 + cu;
    // dH is the layer output's gradient as autograd hands it (bf16), or fp32;
    // row pitch ldh >= Hd: a column slice of a wider gradient (the backward
    // of a feature concat) is read in place, with no gather copy
    nx_dh = dh_bf16 ? bf2f(((const bf16_t*)dH)[row * ldh + j]) : dH[row * ldh + j];
    const float* a = act + row * 5 * Hd + j;
#pragma unroll
    for (int q = 0; q < 5; ++q) nx_a[q] = a[(long)q * Hd];
    nx_cp = 0.f;
    if (fwd_idx > 0) {
      const int tp = reverse ? t + 1 : t - 1;
      nx_cp = cs[((long)tp * B + b0 + cr) * Hd + j];
    }
  };
  if (cell) load_cell(0);
  for (int s = 0; s < T; ++s) {
    const int t = reverse ? s : T - 1 - s;             // backward order
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    if (s > 0) {
      const int tn = reverse ? t - 1 : t + 1;
      const unsigned goff = (unsigned)((((long)tn * B + b0 + (lane & 15)) * 4 * Hd + kb) * 2);
      constexpr int BCH = PL_BCH < KW ? PL_BCH : KW;
#pragma unroll
      for (int h = 0; h < KW; h += BCH) {
        s16x8_t ga[BCH];
#pragma unroll
        for (int u = 0; u < BCH; ++u) ga[u] = pl_ld16(grs, goff + 64 * (h + u));
#pragma unroll
        for (int u = 0; u < BCH; ++u) {
          const int ks = h + u;
          const s16x8_t b = ks < KWR ? wf[ks < KWR ? ks : 0] : wlds[wv][ks >= KWR ? ks - KWR : 0][lane];
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, ga[u]),
                                                        __builtin_bit_cast(bf16x8_t, b), acc, 0, 0, 0);
        }
      }
    }
    const float dhv = nx_dh, cpv = nx_cp;
    float av[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) av[q] = nx_a[q];
#pragma unroll
    for (int r = 0; r < 4; ++r) red[ksl][4 * (lane >> 4) + r][16 * half + (lane & 15)] = acc[r];
    __syncthreads();
    if (cell) {
      float dh = dhv;
#pragma unroll
      for (int k = 0; k < PL_W; ++k) dh += red[k][cr][cu];
      const float i_ = av[0], f_ = av[1], g_ = av[2], o_ = av[3], tc = av[4];
      const float dc = dh * o_ * (1.f - tc * tc) + dc_reg;
      gbuf[cr][cu] = f2bf(dc * g_ * i_ * (1.f - i_));
      gbuf[cr][U + cu] = f2bf(dc * cpv * f_ * (1.f - f_));
      gbuf[cr][2 * U + cu] = f2bf(dc * i_ * (1.f - g_ * g_));
      gbuf[cr][3 * U + cu] = f2bf(dh * tc * o_ * (1.f - o_));
      dc_reg = dc * f_;
    }
    __syncthreads();
    if (wv == 0) {
      // 16 rows x 4 gates x U units of dG_t: (4 x CH) x (64 lanes x 8 B), write-through
#pragma unroll
      for (int u = 0; u < 4 * CH; ++u) {
        const int idx = u * 64 + lane, r = idx / (16 * CH), rem = idx % (16 * CH);
        const int g = rem / (4 * CH), q = rem % (4 * CH);
        const unsigned long long v = *(const unsigned long long*)&gbuf[r][g * U + 4 * q];
        __hip_atomic_store((pl_gu64*)(dG + ((long)t * B + b0 + r) * 4 * Hd + g * Hd + j0 + 4 * q), v,
                           PL_RLX);
      }
      if (s + 1 < T) pl_signal(sync, bt * ns + ut % ns);
    }
    if (cell && s + 1 < T) load_cell(s + 1);   // after the signal's vmcnt(0) drain
    if (s + 1 < T) pl_wait(sync, bt * ns, ns, (unsigned)(s + 1) * (unsigned)(Hd / U / ns), job_err);
  }
}

// Co-residency: `grids` such grids must fit at once (GPU sharing can put
// two GNMT jobs on one device), on the CUs left after `rsv` are set aside
// for kernels that run concurrently with the recurrence and are not ours --
// RCCL's all-reduce of a DDP gang occupies up to one workgroup per channel.
// Passed with every launch by the job's model (GNMT.residency; a process-
// wide setting would let two jobs sharing a device overwrite each other's);
// lstm_seq_residency only sets the default for callers that pass none
// (grids < 0). The occupancy query is cached per kernel.
static int g_pl_grids = 2, g_pl_rsv_cus = 0;
TAM_KNOB(g_pl_grids) TAM_KNOB(g_pl_rsv_cus)
void lstm_seq_residency(int grids, int reserved_cus) {
  g_pl_grids = grids < 1 ? 1 : grids;
  g_pl_rsv_cus = reserved_cus < 0 ? 0 : reserved_cus;
}

static bool pl_fits(const void* kern, int threads, int grid, int grids, int rsv) {
  static std::mutex mu;
  static std::map<const void*, std::pair<int, int>> cap;   // kernel -> (per CU, CUs)
  if (grids < 1) {
    grids = g_pl_grids;
    rsv = g_pl_rsv_cus;
  }
  std::lock_guard<std::mutex> g(mu);
  auto it = cap.find(kern);
  if (it == cap.end()) {
    int per_cu = 0, dev = 0, cus = 0;
    if (!(hipGetDevice(&dev) == hipSuccess &&
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, 0) == hipSuccess))
      per_cu = cus = 0;
    it = cap.emplace(kern, std::make_pair(per_cu, cus)).first;
  }
  const int usable = it->second.first * (it->second.second - (rsv < 0 ? 0 : rsv));
  return grids * grid <= usable;
}

int64_t lstm_persist_timeouts(bool reset) {
  unsigned v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_pl_timeouts), sizeof(v), 0, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  if (reset && v) {
    unsigned z = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pl_timeouts), &z, sizeof(z), 0, hipMemcpyHostToDevice);
  }
  return (int64_t)v;
}

const unsigned* lstm_timeout_word() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_pl_timeouts)) != hipSuccess) return nullptr;
  return (const unsigned*)p;
}

void lstm_seq_spin_limit(int64_t polls) {
  unsigned v = polls <= 0 ? PL_SPIN : (unsigned)polls;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pl_spin), &v, sizeof(v), 0, hipMemcpyHostToDevice);
}

static int g_pl_ch = 0;   // 0: auto (1), 1 / 2: forced
void lstm_seq_policy(int ch) { g_pl_ch = ch; }

// arrival counters per batch tile (1, 2 or 4). Measured (tools/ab_lstm_shards.py,
// GNMT hipGraph step, interleaved): 1 -> 10.95 ms, 2 -> 10.71, 4 -> 10.97. With
// B = 64 (4 batch tiles) a tile's workgroups bt + 4 ut sit on two XCDs under
// round-robin dispatch, split by ut parity: 2 counters = one per XCD
static int g_pl_ns = 2;
TAM_KNOB(g_pl_ns)
TAM_KNOB(g_pl_ch)
void lstm_seq_shards(int ns) { g_pl_ns = (ns == 2 || ns == 4) ? ns : 1; }

static int pl_ch(int Hd) {
  if (g_pl_ch == 1 || g_pl_ch == 2) return g_pl_ch;
  return 1;   // measured: 2 is slower (latency-bound steps: fwd 220 vs 196, bwd 499 vs 318 us/seq)
}

template <int KW, int CH>
static bool pl_fwd(const float* gx, const bf16_t* w_hh, bf16_t* hs, float* cs, float* act, int T, int B,
                   int Hd, int reverse, unsigned* sync, const PLOpts& o, hipStream_t s) {
  const int grid = (B / 16) * (Hd / (16 * CH));
  auto k = lstm_persist_fwd_kernel<KW, CH>;
  if (!pl_fits((const void*)k, 64 * PL_W * CH, grid, o.grids, o.rsv)) return false;
  const int ns = (Hd / (16 * CH)) % g_pl_ns == 0 ? g_pl_ns : 1;
  if (!o.zeroed) zero_async(sync, (size_t)(1 + (B / 16) * ns) * 128, s);   // error flag line + counters
  hipLaunchKernelGGL(k, dim3(grid), dim3(64 * PL_W * CH), 0, s, gx, w_hh, hs, cs, act, T, B, Hd, reverse,
                     sync, ns, o.job_err);
  return true;
}

template <int KW, int CH>
static bool pl_bwd(const float* act, const float* cs, const float* dH, const bf16_t* w_hh, bf16_t* dG, int T,
                   int B, int Hd, int reverse, unsigned* sync, int dh_bf16, int ldh, const PLOpts& o,
                   hipStream_t s) {
  const int grid = (B / 16) * (Hd / (16 * CH));
  auto k = lstm_persist_bwd_kernel<KW, CH>;
  if (!pl_fits((const void*)k, 64 * PL_W * CH, grid, o.grids, o.rsv)) return false;
  const int ns = (Hd / (16 * CH)) % g_pl_ns == 0 ? g_pl_ns : 1;
  if (!o.zeroed) zero_async(sync, (size_t)(1 + (B / 16) * ns) * 128, s);   // error flag line + counters
  hipLaunchKernelGGL(k, dim3(grid), dim3(64 * PL_W * CH), 0, s, act, cs, dH, w_hh, dG, T, B, Hd, reverse,
                     sync, ns, dh_bf16, ldh, o.job_err);
  return true;
}

bool lstm_seq_forward(const float* gx, const bf16_t* w_hh, bf16_t* hs, float* cs, float* act, int T,
                      int B, int Hd, int reverse, unsigned* sync, hipStream_t s, const PLOpts& o) {
  if (T < 1 || B % 16 != 0 || Hd % 256 != 0 || 8 % (B / 16) != 0) return false;
  const int kw = Hd / (32 * PL_W), ch = pl_ch(Hd);
#define PL_F(KWV)                                                                                    \
  case KWV:                                                                                          \
    return ch == 2 ? pl_fwd<KWV, 2>(gx, w_hh, hs, cs, act, T, B, Hd, reverse, sync, o, s)           \
                   : pl_fwd<KWV, 1>(gx, w_hh, hs, cs, act, T, B, Hd, reverse, sync, o, s);
  switch (kw) {
    PL_F(1)
    PL_F(2)
    PL_F(4)
    default: return false;
  }
#undef PL_F
}

bool lstm_seq_backward(const float* act, const float* cs, const float* dH, const bf16_t* w_hh, bf16_t* dG,
                       int T, int B, int Hd, int reverse, unsigned* sync, int dh_bf16, int ldh, hipStream_t s,
                       const PLOpts& o) {
  if (T < 1 || B % 16 != 0 || Hd % 256 != 0 || 8 % (B / 16) != 0 || ldh < Hd) return false;
  const int kw = 4 * Hd / (32 * PL_W), ch = pl_ch(Hd);
#define PL_B(KWV)                                                                                    \
  case KWV:                                                                                          \
    return ch == 2 ? pl_bwd<KWV, 2>(act, cs, dH, w_hh, dG, T, B, Hd, reverse, sync, dh_bf16, ldh, o, s)  \
                   : pl_bwd<KWV, 1>(act, cs, dH, w_hh, dG, T, B, Hd, reverse, sync, dh_bf16, ldh, o, s);
  switch (kw) {
    PL_B(4)
    PL_B(8)
    PL_B(16)
    default: return false;
  }
#undef PL_B
}

static int lgrid(long n) { long b = (n + 255) / 256; if (b > 2048) b = 2048; return (int)(b < 1 ? 1 : b); }

void lstm_cell_forward(const float* gates, const float* c_prev, float* c_out, bf16_t* h_out,
                       float* h_out_f32, float* act_cache, int B, int Hd, hipStream_t s) {
  hipLaunchKernelGGL(lstm_fwd_kernel, dim3(lgrid((long)B * Hd)), dim3(256), 0, s, gates, c_prev,
                     c_out, h_out, h_out_f32, act_cache, B, Hd);
}

void lstm_cell_backward(const float* act_cache, const float* c_prev, const float* c_out,
                        const float* dh, const float* dc_next, float* dgates, float* dc_prev,
                        bf16_t* dgates_bf16, int B, int Hd, hipStream_t s) {
  (void)c_out;
  hipLaunchKernelGGL(lstm_bwd_kernel, dim3(lgrid((long)B * Hd)), dim3(256), 0, s, act_cache, c_prev,
                     dh, dc_next, dgates, dc_prev, dgates_bf16, B, Hd);
}

}  // namespace tam
