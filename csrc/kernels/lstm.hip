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
