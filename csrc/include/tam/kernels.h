// tiresias_amd — host launch API for the non-GEMM kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "tam/common.h"

namespace tam {

// BatchNorm (NHWC rows=M=N*H*W, C channels, C % 8 == 0, C <= 2048).
// Statistics: fp64 sums[BN_SHARDS][2C] (norm.hip), zeroed by the caller;
// sums_ready: the producer (a conv epilogue) already accumulated them -- no
// reduction pass here (else one pass adds them with sharded fp64 atomics).
// ymask (relu BNs): forward stores 1 bit per output (y > 0, byte (r*C+c)/8,
// bit c%8); backward given ymask (and y == nullptr) masks with the bits
// instead of re-reading the bf16 y -- 1/16 of the bytes.
constexpr int BN_MAX_BLOCKS = 512;
constexpr int LN_MAX_BLOCKS = 512;
constexpr int COLSUM_MAX_BLOCKS = 256;
// out[c] = sum over nblk partial rows part[b][c] (width W): fp64 store, or fp32
// accumulate into out0[c] (c < split) / out1[c - split]
void col_reduce_f64(const float* part, int nblk, int W, double* out, hipStream_t s);
constexpr int CR_BATCH_MAX = 48;   // column reduces per batched launch (kernel-argument budget)
// col_reduce_acc over n (part, nblk, W, out0, out1, split) entries in one launch per 48
void col_reduce_acc_batch(const float* const* part, const int* nblk, const int* W, float* const* out0,
                          float* const* out1, const int* split, int n, hipStream_t s);
void col_reduce_acc(const float* part, int nblk, int W, float* out0, float* out1, int split,
                    hipStream_t s);
void bn_forward(const bf16_t* x, const bf16_t* res, bf16_t* y, long M, int C, float eps,
                float momentum, const float* gamma, const float* beta, float* run_mean,
                float* run_var, float* save_mean, float* save_rstd, int relu, double* sums,
                int sums_ready, uint8_t* ymask, hipStream_t s);
void bn_infer(const bf16_t* x, const bf16_t* res, bf16_t* y, long M, int C, const float* scale,
              const float* shift, int relu, hipStream_t s);
// batched conv weight re-layout [K][RS][C] -> [C][RS][K] (one launch)
struct WTEntry {
  const bf16_t* w;
  bf16_t* wt;
  int K, RS, C, tile0;
};
constexpr int WT_MAX = 64;
struct WTBatch {
  int n;
  WTEntry e[WT_MAX];
};
void conv_weight_t_batch(WTBatch& b, hipStream_t s);
// addend (optional): a second upstream gradient of y summed into dy on load
// (the residual branch's, so autograd never materialises the sum).
// sums: fp64 [BN_SHARDS][2C] sum(d) | sum(d*xhat); sums_ready: accumulated
// by the consumer conv's dgrad epilogue (Epi::bnx, which also applied the
// ReLU mask)
void bn_backward(const bf16_t* dy, const bf16_t* addend, const bf16_t* y, const bf16_t* x, const float* mean,
                 const float* rstd, const float* gamma, long M, int C, int relu, bf16_t* dx,
                 bf16_t* dres, float* dgamma, float* dbeta, double* sums, int sums_ready,
                 const uint8_t* ymask, hipStream_t s);

// LayerNorm over last dim D (D % 8 == 0, D <= 2048)
// addend (optional): LN of (x + addend), the bf16 sum also stored to sum_out
// (a residual add fused into the next pre-LN)
void ln_forward(const bf16_t* x, const float* g, const float* b, bf16_t* y, float* mean,
                float* rstd, long rows, int D, float eps, hipStream_t s, const bf16_t* addend = nullptr,
                bf16_t* sum_out = nullptr);
// dx = LN-backward(dy) (+ addend, the fused gradient of a skip connection)
void ln_backward(const bf16_t* dy, const bf16_t* x, const float* g, const float* mean,
                 const float* rstd, bf16_t* dx, const bf16_t* addend, float* dg, float* db,
                 float* ws, long rows, int D, hipStream_t s);
// the same without the column reduce: per-block partial dgamma | dbeta rows
// in ws; returns their count (col_reduce_acc finishes, e.g. on a side stream)
int ln_backward_partial(const bf16_t* dy, const bf16_t* x, const float* g, const float* mean,
                        const float* rstd, bf16_t* dx, const bf16_t* addend, float* ws, long rows, int D,
                        hipStream_t s);

// pooling
void maxpool_forward(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int P,
                     int Q, int R, int S, int st, int pad, hipStream_t s);
void maxpool_k3s2_policy(int p);   // 1: 3x3/s2/p1 backward kernel (default), 0: generic
void maxpool_backward(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C,
                      int P, int Q, int R, int S, int st, int pad, hipStream_t s);
void avgpool_forward(const bf16_t* x, bf16_t* y, int N, int HW, int C, hipStream_t s);
void avgpool_backward(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t s);

// fused softmax cross-entropy (forward + backward)
// tm_b > 0: logits rows time-major (r = s * tm_b + b), labels [tm_b][S]
void softmax_xent(const bf16_t* logits, const long* labels, bf16_t* dlogits, float* loss_rows,
                  long rows, int V, float smoothing, float grad_scale, long ignore_index,
                  hipStream_t s, long tm_b = 0);
// out[0] = scale * sum(x[0..n))
void sum_scale(const float* x, long n, float* out, float scale, hipStream_t s);

// embedding
// V = table rows: ids outside [0, V) read zero rows / take no gradient;
// tm_b > 0: ids [tm_b][S], rows of out / dout time-major (t = s * tm_b + b)
// pos (optional [pos_rows][D]): + pos[position of t] (batch-major: t % pos_rows)
void embedding_forward(const bf16_t* table, const long* ids, bf16_t* out, long T, int D,
                       float scale, hipStream_t s, long V, long tm_b = 0, const bf16_t* pos = nullptr,
                       long pos_rows = 0);
void embedding_backward(const bf16_t* dout, const long* ids, float* gtable, long T, int D,
                        float scale, hipStream_t s, long V, long tm_b = 0);

// row-block copies / sums (bf16): up to 4 jobs per launch, each
// out[r][0..C) = sum_q in_q[r][0..C) over n_in <= 4 pitched inputs
struct RowJob {
  const bf16_t* in[4];
  long ld_in[4];
  bf16_t* out;
  long ld_out;
  int C, n_in;
};
struct RowJobs {
  RowJob job[4];
};
void rows_sum(const RowJobs& jb, int njobs, long R, hipStream_t s);

// misc
// out[c] += sum_r x[r][c]; ws: COLSUM_MAX_BLOCKS * C floats (C % 8 == 0 path)
void colsum(const bf16_t* x, float* out, float* ws, long R, int C, hipStream_t s);
void colsum_policy(int p);   // 0 auto, 1 partial rows + reduce, 2 atomics (A/B)
void relu_backward(const bf16_t* dy, const bf16_t* y, bf16_t* dx, long n, hipStream_t s);
void add_bf16(const bf16_t* a, const bf16_t* b, bf16_t* y, long n, hipStream_t s);
void cast_f32_bf16(const float* x, bf16_t* y, long n, hipStream_t s);

// optimizers over flat arenas (n % 4 == 0)
void optim_grid(int blocks);   // grid cap of the optimizer launches (A/B; 0 = one block per CU)
void sgd_step(float* w, float* g, float* mom, bf16_t* wb, long n, float lr, float momentum,
              float wd, float gscale, int nesterov, int zero_grad, hipStream_t s,
              const unsigned* guard = nullptr, long zero_from = 0, long wd_until = -1);
void optim_variant(int v);   // streaming optimizer variants (optim.hip), 0 = baseline
void adam_step(float* w, float* g, float* m, float* v, bf16_t* wb, long n, float lr, float b1,
               float b2, float eps, float wd, int step, float gscale, int zero_grad,
               hipStream_t s, const unsigned* guard = nullptr, long zero_from = 0, long wd_until = -1);

// fused attention (bf16, head_dim 64): element (b, s, h, d) at b * *_bstride +
// s * *_stride + 64 h + d (batch-major [B][S][H][64], or a time-major
// [S][B][H][64] tensor with bstride = H*64 per batch row)
void attn_forward(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B,
                  int H, int Sq, int Sk, long q_stride, long kv_stride, long o_stride, long q_bstride,
                  long kv_bstride, long o_bstride, int causal, float scale, const int* kv_len, hipStream_t s);
void attn_short_policy(int p);   // 1: Sk <= 128 backward in one fused launch (default)
void attn_backward(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o,
                   const bf16_t* dout, const float* lse, bf16_t* dq, bf16_t* dk, bf16_t* dv,
                   float* dq_acc, float* delta, int B, int H, int Sq, int Sk, long q_stride,
                   long kv_stride, long o_stride, long q_bstride, long kv_bstride, long o_bstride, int causal,
                   float scale, const int* kv_len, hipStream_t s);

// LSTM cell pointwise (gates = x W_ih^T + h W_hh^T + b precomputed, fp32)
void lstm_cell_forward(const float* gates, const float* c_prev, float* c_out, bf16_t* h_out,
                       float* h_out_f32, float* act_cache, int B, int Hd, hipStream_t s);
// fused forward timestep (B % 16 == 0, Hd % 256 == 0): h_out/c_out/act for one t
void lstm_step_forward(const float* gx, const bf16_t* w_hh, const bf16_t* h_prev, const float* c_prev,
                       float* c_out, bf16_t* h_out, float* act, int B, int Hd, hipStream_t s);
// persistent whole-sequence recurrence (lstm.hip); false = shape / residency
// not supported (the caller runs the per-step path). sync: int32 words,
// [0] error flag, [32 * (bt + 1)] per-batch-tile counters (zeroed here).
// PLOpts: per-launch co-residency rule (grids that must fit at once, CUs
// reserved for foreign kernels; grids < 0: the lstm_seq_residency default)
// and the launching job's own timeout word (nullable).
struct PLOpts {
  int grids = -1, rsv = 0;
  unsigned* job_err = nullptr;
  int zeroed = 0;    // 1: the caller zeroed the sync words (one fill for a whole step's launches)
};
bool lstm_seq_forward(const float* gx, const bf16_t* w_hh, bf16_t* hs, float* cs, float* act, int T,
                      int B, int Hd, int reverse, unsigned* sync, hipStream_t s, const PLOpts& o = PLOpts());
// dH: [T][B] rows of Hd values at row pitch ldh (>= Hd; elements)
bool lstm_seq_backward(const float* act, const float* cs, const float* dH, const bf16_t* w_hh, bf16_t* dG,
                       int T, int B, int Hd, int reverse, unsigned* sync, int dh_bf16, int ldh, hipStream_t s,
                       const PLOpts& o = PLOpts());
// the job's guard word after its optimizer step: err[0] != 0 (a timed-out
// barrier this step; the optimizer skipped the update) -> err[1] += 1, err[0] = 0
void lstm_guard_step(unsigned* err, hipStream_t s);
// unit halves per persistent workgroup: 0 auto, 1 (16 units) or 2 (32 units)
void lstm_seq_policy(int ch);
void lstm_seq_shards(int ns);   // arrival counters per batch tile (1, 2, 4)
void lstm_seq_residency(int grids, int reserved_cus);   // co-residency rule of the persistent grids
int64_t lstm_persist_timeouts(bool reset);              // sticky barrier-timeout count (device)
void lstm_seq_spin_limit(int64_t polls);                // barrier poll bound (<= 0: default)
const unsigned* lstm_timeout_word();                     // device address of the timeout counter
void lstm_cell_backward(const float* act_cache, const float* c_prev, const float* c_out,
                        const float* dh, const float* dc_next, float* dgates, float* dc_prev,
                        bf16_t* dgates_bf16, int B, int Hd, hipStream_t s);

}  // namespace tam
