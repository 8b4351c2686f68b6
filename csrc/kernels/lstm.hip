// tiresias_amd — fused LSTM cell pointwise (GNMT). The gate pre-activations
// G = X W_ih^T + h W_hh^T + b are produced by the MFMA GEMM (fp32 output,
// the x-part for all timesteps in one GEMM, the h-part accumulated per step);
// this kernel does every elementwise op of the cell in one pass and caches the
// activations the backward needs. Gate order: i, f, g, o.
#include "tam/common.h"
#include "tam/kernels.h"

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
