#include <array>
// tiresias_amd — torch custom-op registration for the HIP kernel library.
// Every op validates device / dtype / layout and fails loudly; all launches go
// to the caller's current HIP stream (so they compose with RCCL side streams
// and hipGraph capture).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <functional>
#include <map>
#include <mutex>
#include <sstream>
#include <tuple>
#include <vector>

#include "tam/kernels.h"
#include "tam/launch.h"
#include "tam/gemm8p.h"

using at::Tensor;
using c10::optional;

namespace {

hipStream_t cur_stream(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check_dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.defined(), "tam: ", name, " is undefined");
  TORCH_CHECK(t.is_cuda(), "tam: ", name, " must be a GPU tensor (HIP), got ", t.device());
}
void check_bf16(const Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "tam: ", name, " must be bfloat16, got ",
              t.scalar_type());
}
void check_f32(const Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat, "tam: ", name, " must be float32, got ", t.scalar_type());
}
void check_contig(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_contiguous(), "tam: ", name, " must be contiguous");
}
const tam::bf16_t* bp(const Tensor& t) { return reinterpret_cast<const tam::bf16_t*>(t.data_ptr()); }
tam::bf16_t* bpm(const Tensor& t) { return reinterpret_cast<tam::bf16_t*>(t.data_ptr()); }
template <class T>
T* opt_ptr(const optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

// ------------------------------------------------------------------ GEMM
// Measured routing for PLAIN GEMMs (no fused relu / relu-mask epilogue): the
// hand-written MFMA kernel vs hipBLASLt reached through ATen (mm / addmm with
// an fp32 out_dtype, so fp32 grad accumulation stays one library call). Each
// (shape, majorities, epilogue) key is timed ONCE on scratch output with HIP
// events, outside graph capture, and cached per process; fused epilogues and
// small problems always take the MFMA kernel. Policy: -1 measured (default),
// 0 MFMA only, 1 library whenever eligible.
using GemmKey = std::tuple<int64_t, int64_t, int64_t, bool, bool, int64_t, bool, bool>;
std::map<GemmKey, int> g_route;          // 0 = igemm/gemm256, 1 = library, 2 = LDS-DMA GEMM
std::map<GemmKey, std::array<float, 4>> g_route_ms;   // measured ms per path
std::mutex g_route_mu;
// hipBLASLt for PLAIN GEMMs: 0 (default since round 6) never -- every GEMM
// of every model runs on our MFMA kernels, the routing only picks among them
// (tile, slab split, stream-K, igemm); -1 measured per-shape routing that may
// pick the library where it timed > 5 % faster (A/B against the library
// only, TAM_GEMM_LIB=-1); 1 library wherever eligible (A/B only).
// Round 5 had made -1 the default (Transformer -0.24 ms, GNMT -0.21 ms from
// 15 of 51 plain shapes on the library); the north star wants hand-written
// kernels on the hot path, so the library is an A/B reference now.
int g_lib_policy = [] {
  const char* e = getenv("TAM_GEMM_LIB");
  return e ? atoi(e) : 0;
}();
extern int g_dma_policy;
int g_forced = 0;   // tile/split forced for tuning: never route to the library
TAM_KNOB(g_lib_policy) TAM_KNOB(g_forced)

void run_mfma(const Tensor& a, bool ak, const Tensor& b, bool bk, int64_t M, int64_t N, int64_t K,
              const tam::Epi& ep, bool allow_split, int path = -1) {
  if (path < 0)
    tam::gemm(bp(a), a.stride(0), ak, bp(b), b.stride(0), bk, (int)M, (int)N, (int)K, ep,
              allow_split, cur_stream(a));
  else
    tam::gemm_select(bp(a), a.stride(0), ak, bp(b), b.stride(0), bk, (int)M, (int)N, (int)K, ep,
                     allow_split, cur_stream(a), path);
}

void run_lib(const Tensor& a, bool ak, const Tensor& b, bool bk, const Tensor& c, int64_t mode,
             const optional<Tensor>& bias) {
  const Tensor Ae = ak ? a : a.t();   // [M][K]
  const Tensor Be = bk ? b.t() : b;   // [K][N]
  Tensor out = c;
  if (mode == 1) {
    at::addmm_out(out, c, Ae, Be, at::kFloat, 1, 1);
  } else if (bias.has_value() && bias->defined()) {
    at::addmm_out(out, *bias, Ae, Be);
  } else if (c.scalar_type() == at::kFloat) {
    at::mm_out(out, Ae, Be, at::kFloat);
  } else {
    at::mm_out(out, Ae, Be);
  }
}

// 256^2 all-layout kernel; slab split-K (fp32 workspace, one reduce pass,
// any output dtype) when its tile grid underfills the chip
// tile / sp < 0: the heuristics (gemm8p_tile, gemm8p_slab_splits); the
// measured routing passes the (tile, splits) it timed best
// sp == 0 (tile 256): the stream-K schedule; g_sk_force: the heuristic
// configuration becomes stream-K wherever eligible (tests)
int g_sk_force = 0;
TAM_KNOB(g_sk_force)
void run_p8(const Tensor& a, bool ak, const Tensor& b, bool bk, int64_t M, int64_t N, int64_t K,
            const tam::Epi& ep, bool allow_split, int tile = -1, int sp = -1) {
  if ((sp == 0 || (g_sk_force && tile < 0)) &&
      tam::gemm8p_sk_ok(ak, bk, (int)M, (int)N, (int)K, a.stride(0), b.stride(0))) {
    Tensor ws = at::empty({tam::gemm8p_sk_ws_floats((int)M, (int)N, (int)K)}, a.options().dtype(at::kFloat));
    tam::gemm8p_streamk(bp(a), a.stride(0), ak, bp(b), b.stride(0), bk, (int)M, (int)N, (int)K, ep,
                        ws.data_ptr<float>(), cur_stream(a));
    return;
  }
  if (sp == 0) sp = -1;
  const bool explicit_cfg = tile > 0;
  if (tile < 0) tile = tam::gemm8p_tile((int)M, (int)N, (int)K);
  if (!tam::gemm8p_tile_ok(tile, ak)) tile = 128;
  if (sp < 0) sp = tam::gemm8p_slab_splits((int)M, (int)N, (int)K, tile);
  if (sp > 1 && ep.ldc >= N) {
    Tensor ws = at::empty({sp, M, N}, a.options().dtype(at::kFloat));
    tam::gemm8p_splitk(bp(a), a.stride(0), ak, bp(b), b.stride(0), bk, (int)M, (int)N, (int)K, ep, sp,
                       ws.data_ptr<float>(), cur_stream(a), tile);
    return;
  }
  if (explicit_cfg)
    tam::launch_gemm8p(bp(a), a.stride(0), ak, bp(b), b.stride(0), bk, (int)M, (int)N, (int)K, ep, 1,
                       cur_stream(a), tile);
  else
    run_mfma(a, ak, b, bk, M, N, K, ep, allow_split, 3);
}
void run_skinny(const Tensor& a, const Tensor& b, bool bk, int64_t M, int64_t N, int64_t K, const tam::Epi& ep) {
  const int sp = tam::gemm_skinny_splits((int)M, (int)N, (int)K);
  Tensor ws;
  if (sp > 1) ws = at::empty({sp, M, N}, a.options().dtype(at::kFloat));
  tam::gemm_skinny(bp(a), a.stride(0), bp(b), b.stride(0), bk, (int)M, (int)N, (int)K, ep, sp,
                   sp > 1 ? ws.data_ptr<float>() : nullptr, cur_stream(a));
}
// measured (tile, splits) of the p8 route per key
std::map<GemmKey, std::pair<int, int>> g_p8_cfg;

float time_ms(hipStream_t s, const std::function<void()>& fn) {
  fn();   // warm (library heuristics / our first launch)
  hipEvent_t e0, e1;
  TAM_HIP_CHECK(hipEventCreate(&e0));
  TAM_HIP_CHECK(hipEventCreate(&e1));
  TAM_HIP_CHECK(hipEventRecord(e0, s));
  for (int i = 0; i < 3; ++i) fn();
  TAM_HIP_CHECK(hipEventRecord(e1, s));
  TAM_HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  TAM_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  TAM_HIP_CHECK(hipEventDestroy(e0));
  TAM_HIP_CHECK(hipEventDestroy(e1));
  return ms / 3.f;
}

// routing (tuned per shape) + launch of one GEMM whose epilogue is set up
void gemm_dispatch(const Tensor& a, bool a_kmajor, const Tensor& b, bool b_kmajor, const Tensor& c,
                   int64_t mode, const optional<Tensor>& bias, bool relu, double alpha, bool allow_split,
                   int64_t M, int64_t N, int64_t K, const tam::Epi& ep);

// the bias-gradient fusion (Epi::colsum_a) runs on the register-staged igemm
// only: fuse when that is the routed path, or when it is at most this much
// slower than the routed one (a separate column-sum pass costs ~5-9 us on the
// Transformer's shapes, profiles/r3/s3/ab_colsum.json)
constexpr float COLSUM_FUSE_SLACK_MS = 0.005f;

// a: (M,K) if a_kmajor else (K,M); b: (N,K) if b_kmajor else (K,N); c: (M,N)
// colsum (M-major A only): colsum[m] += sum_k A[k][m] (fp32) -- the bias
// gradient of a Linear layer whose weight gradient this GEMM computes
void gemm_op(const Tensor& a, bool a_kmajor, const Tensor& b, bool b_kmajor, const Tensor& c,
             int64_t mode, const optional<Tensor>& bias, bool relu, const optional<Tensor>& mask,
             double alpha, bool allow_split, const optional<Tensor>& colsum) {
  check_bf16(a, "a");
  check_bf16(b, "b");
  check_dev(c, "c");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "tam.gemm: 2-D operands required");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && c.stride(1) == 1,
              "tam.gemm: inner dim must be unit-stride");
  const int64_t M = a_kmajor ? a.size(0) : a.size(1);
  const int64_t K = a_kmajor ? a.size(1) : a.size(0);
  const int64_t N = b_kmajor ? b.size(0) : b.size(1);
  const int64_t Kb = b_kmajor ? b.size(1) : b.size(0);
  TORCH_CHECK(K == Kb, "tam.gemm: K mismatch ", K, " vs ", Kb);
  TORCH_CHECK(c.size(0) == M && c.size(1) == N, "tam.gemm: C shape mismatch");
  TORCH_CHECK((!a_kmajor && !b_kmajor) || K % 8 == 0,
              "tam.gemm: K must be a multiple of 8 for a K-major operand");
  TORCH_CHECK(a_kmajor || M % 8 == 0, "tam.gemm: M-major A needs M % 8 == 0");
  TORCH_CHECK(b_kmajor || N % 8 == 0, "tam.gemm: N-major B needs N % 8 == 0");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0, "tam.gemm: 16-byte aligned rows needed");
  tam::Epi ep;
  ep.c = c.data_ptr();
  ep.ldc = c.stride(0);
  ep.c_f32 = c.scalar_type() == at::kFloat;
  TORCH_CHECK(ep.c_f32 || c.scalar_type() == at::kBFloat16, "tam.gemm: C must be f32 or bf16");
  ep.mode = (int)mode;
  TORCH_CHECK(mode == 0 || mode == 1 || (mode == 2 && ep.c_f32), "tam.gemm: bad mode");
  if (bias.has_value() && bias->defined()) {
    check_bf16(*bias, "bias");
    TORCH_CHECK(bias->numel() == N, "tam.gemm: bias size");
  }
  ep.bias = bias.has_value() && bias->defined() ? bp(*bias) : nullptr;
  ep.relu = relu;
  if (mask.has_value() && mask->defined()) {
    check_bf16(*mask, "mask");
    TORCH_CHECK(mask->dim() == 2 && mask->size(0) == M && mask->size(1) == N && mask->stride(1) == 1,
                "tam.gemm: mask shape");
    ep.mask = bp(*mask);
    ep.ldm = mask->stride(0);
  }
  ep.alpha = (float)alpha;
  if (colsum.has_value() && colsum->defined()) {
    TORCH_CHECK(!a_kmajor, "tam.gemm: colsum needs an M-major A");
    check_f32(*colsum, "colsum");
    TORCH_CHECK(colsum->numel() == M && colsum->is_contiguous(), "tam.gemm: colsum size");
    const GemmKey key{M, N, K, a_kmajor, b_kmajor, mode, (bool)ep.c_f32, bias.has_value() && bias->defined()};
    bool fuse = false;
    {
      std::lock_guard<std::mutex> g(g_route_mu);
      auto it = g_route.find(key);
      if (it != g_route.end()) {
        const auto t = g_route_ms[key];
        fuse = it->second == 0 || t[0] <= t[it->second] + COLSUM_FUSE_SLACK_MS;
      }
    }
    // shapes gemm_dispatch never tunes go straight to the igemm anyway
    const double mnk = (double)M * N * K;
    const bool tuned = (g_lib_policy != 0 && mnk >= (double)(1 << 27)) ||
                       (g_dma_policy == 1 && K % 64 == 0 && mnk >= (double)(1 << 24)) ||
                       (tam::gemm8p_policy_mode() == 1 && mnk >= (double)(1 << 27) &&
                        tam::gemm8p_ok(a_kmajor, b_kmajor, (int)M, (int)N, (int)K, a.stride(0), b.stride(0)));
    if (!tuned) fuse = true;
    // route 0 of a big shape IS the LDS-DMA kernel (gemm_select's size rule),
    // which the fusion would trade for the igemm: never worth it
    if (tam::gemm_select_big_p8(a_kmajor, b_kmajor, (int)M, (int)N, (int)K, a.stride(0), b.stride(0)))
      fuse = false;
    if (fuse && !g_forced && tam::gemm8p_policy_mode() != 3 && g_dma_policy != 2) {
      ep.colsum_a = colsum->data_ptr<float>();
      run_mfma(a, a_kmajor, b, b_kmajor, M, N, K, ep, allow_split, 0);
      return;
    }
    // not fused (first, tuning call of a shape, or a faster non-igemm route):
    // the GEMM as routed, then the column sums as their own pass over A
    gemm_dispatch(a, a_kmajor, b, b_kmajor, c, mode, bias, relu, alpha, allow_split, M, N, K, ep);
    Tensor ws = at::empty({M % 8 == 0 ? (int64_t)tam::COLSUM_MAX_BLOCKS * M : 1}, a.options().dtype(at::kFloat));
    tam::colsum(bp(a), colsum->data_ptr<float>(), ws.data_ptr<float>(), K, (int)M, cur_stream(a));
    return;
  }
  gemm_dispatch(a, a_kmajor, b, b_kmajor, c, mode, bias, relu, alpha, allow_split, M, N, K, ep);
}

void gemm_dispatch(const Tensor& a, bool a_kmajor, const Tensor& b, bool b_kmajor, const Tensor& c,
                   int64_t mode, const optional<Tensor>& bias, bool relu, double alpha, bool allow_split,
                   int64_t M, int64_t N, int64_t K, const tam::Epi& ep) {
  const bool has_bias = ep.bias != nullptr;
  const bool lib_ok = g_lib_policy != 0 && !g_forced && !relu && ep.mask == nullptr && alpha == 1.0 &&
                      (mode == 0 || (mode == 1 && ep.c_f32)) && !(has_bias && ep.c_f32) &&
                      (double)M * N * K >= (double)(1 << 27) && M >= 16 && N >= 16;
  // gemm8p policy 3: the 256^2 kernel with slab split-K wherever eligible (tests)
  if (tam::gemm8p_policy_mode() == 3 &&
      tam::gemm8p_ok(a_kmajor, b_kmajor, (int)M, (int)N, (int)K, a.stride(0), b.stride(0))) {
    run_p8(a, a_kmajor, b, b_kmajor, M, N, K, ep, allow_split);
    return;
  }
  // skinny M (<= 64, a batch-sized activation times a weight of >= 1 Mi
  // elements): the weight-streaming kernel, split-K over every CU
  if (!g_forced && mode != 2 && (double)N * K >= (double)(1 << 20) &&
      tam::gemm_skinny_ok(a_kmajor, b_kmajor, (int)M, (int)N, (int)K, a.stride(0), b.stride(0))) {
    run_skinny(a, b, b_kmajor, M, N, K, ep);
    return;
  }
  // our two kernels are both candidates for every shape the DMA GEMM accepts
  if (g_dma_policy == 2) {
    run_mfma(a, a_kmajor, b, b_kmajor, M, N, K, ep, allow_split, 2);
    return;
  }
  const bool dma_ok = g_dma_policy == 1 && !g_forced && K % 64 == 0 &&
                      (double)M * N * K >= (double)(1 << 24);
  const bool p8_ok = !g_forced && tam::gemm8p_policy_mode() == 1 &&
                     tam::gemm8p_ok(a_kmajor, b_kmajor, (int)M, (int)N, (int)K, a.stride(0), b.stride(0)) &&
                     (double)M * N * K >= (double)(1 << 27);
  if (g_lib_policy == 1 && lib_ok) {
    run_lib(a, a_kmajor, b, b_kmajor, c, mode, bias);
    return;
  }
  if (!lib_ok && !dma_ok && !p8_ok) {
    run_mfma(a, a_kmajor, b, b_kmajor, M, N, K, ep, allow_split);
    return;
  }
  const GemmKey key{M, N, K, a_kmajor, b_kmajor, mode, (bool)ep.c_f32,
                    has_bias || relu || ep.mask != nullptr};
  int route = -1;
  {
    std::lock_guard<std::mutex> g(g_route_mu);
    auto it = g_route.find(key);
    if (it != g_route.end()) route = it->second;
  }
  if (route < 0) {
    hipStream_t s = cur_stream(a);
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    TAM_HIP_CHECK(hipStreamIsCapturing(s, &cap));
    if (cap != hipStreamCaptureStatusNone) {
      run_mfma(a, a_kmajor, b, b_kmajor, M, N, K, ep, allow_split);   // never tune in a graph
      return;
    }
    // time every candidate on a scratch output so an accumulating C is untouched
    Tensor scratch = at::empty_like(c);
    tam::Epi es = ep;
    es.c = scratch.data_ptr();
    es.ldc = scratch.stride(0);
    std::array<float, 4> t{1e30f, 1e30f, 1e30f, 1e30f};
    std::vector<std::pair<int, int>> cands;
    if (p8_ok) {
      // both tiles, each with its slab split (and the 256^2 tile also with
      // twice that split, and with the largest split that keeps the grid to
      // one wave of 256 blocks): the heuristics alone left 3200x2048x32000 on
      // an unsplit 128^2 grid at ~550 TF/s (256^2 x 2 slabs: ~770,
      // profiles/r2/gemm_deepk.json)
      for (int tl : {256, 128}) {
        const int sp = tam::gemm8p_slab_splits((int)M, (int)N, (int)K, tl);
        cands.push_back({tl, sp});
        if (tl == 256 && sp > 1 && sp * 2 <= 16 && K / 64 / (sp * 2) >= 8) cands.push_back({tl, sp * 2});
        const long t256 = (long)((M + 255) / 256) * ((N + 255) / 256);
        const int one_wave = (int)(256 / t256);
        if (tl == 256 && t256 < 150 && one_wave >= 2 && one_wave != sp && one_wave != 2 * sp &&
            K / 64 / one_wave >= 8)
          cands.push_back({tl, one_wave > 16 ? 16 : one_wave});
        if (tl == 256 && sp == 1 && t256 < 150 && K / 64 >= 32 && one_wave != 2) cands.push_back({tl, 2});
        // deep K over few tiles: the slice count whose block total lands just
        // under a whole number of waves (3200x2048x32000: 104 tiles x 7 = 728
        // blocks = 0.95 of 3 waves, 522 vs 538 us at 2 slices,
        // profiles/r4/streamk_vs_splitk.json)
        if (tl == 256 && t256 < 150 && K / 64 >= 256) {
          int best_sp = 0;
          double best_fill = 0.0;
          for (int q = 3; q <= 16 && K / 64 / q >= 16; ++q) {
            const long blocks = t256 * q;
            const double fill = (double)blocks / (double)(((blocks + 255) / 256) * 256);
            if (fill > best_fill + 1e-9) { best_fill = fill; best_sp = q; }
          }
          if (best_sp && best_sp != sp && best_sp != 2 * sp) cands.push_back({tl, best_sp});
        }
      }
      // 64x128 (K-major A): the N = 512 projections (4096 x 512 = 256 tiles,
      // one per CU) that neither square tile fills
      // (a single-barrier schedule of the 64x128 / 128^2 tiles -- all
      // fragments of K-tile t+1 read under the MFMAs of t, four LDS stages --
      // measured no faster on these shapes and was removed: profiles/r6/
      // gemm_small_tiles.md)
      if (a_kmajor && (M + 63) / 64 * ((N + 127) / 128) >= 128) {
        const int s = tam::gemm8p_slab_splits((int)M, (int)N, (int)K, 64);
        cands.push_back({64, 1});
        if (s > 1) cands.push_back({64, s});
        // ...and with the block's K range over two wave groups (two waves
        // per SIMD at one block per CU, no slab pass): tile code 65
        if ((K / 64) % 2 == 0) cands.push_back({65, 1});
      }
      // 128^2 with the two K groups (tile code 129) where the 128^2 grid is
      // at most one block per CU: GNMT's 3200 x 1024 products (200 tiles)
      if (a_kmajor && (M + 127) / 128 * ((N + 127) / 128) <= 256 && (K / 64) % 2 == 0 && K / 64 >= 8)
        cands.push_back({129, 1});
      if (tam::gemm8p_sk_ok(a_kmajor, b_kmajor, (int)M, (int)N, (int)K, a.stride(0), b.stride(0)))
        cands.push_back({256, 0});   // stream-K
    }
    // two interleaved rounds, best of each: a single timing taken while other
    // streams still drain work (the first eager steps) can be off by 40 %
    std::pair<int, int> p8c{-1, -1};
    for (int round = 0; round < 2; ++round) {
      t[0] = std::min(t[0], time_ms(s, [&] { run_mfma(a, a_kmajor, b, b_kmajor, M, N, K, es, allow_split, 0); }));
      for (const auto& c : cands) {
        const float ms = time_ms(s, [&] { run_p8(a, a_kmajor, b, b_kmajor, M, N, K, es, allow_split, c.first,
                                                 c.second); });
        if (ms < t[3]) { t[3] = ms; p8c = c; }
      }
      if (dma_ok)
        t[2] = std::min(t[2], time_ms(s, [&] { run_mfma(a, a_kmajor, b, b_kmajor, M, N, K, es, allow_split, 2); }));
      if (lib_ok && round == 0) {
        try {
          t[1] = time_ms(s, [&] { run_lib(a, a_kmajor, b, b_kmajor, scratch, mode, bias); });
        } catch (const std::exception&) {
          t[1] = 1e30f;   // library path unsupported for this dtype combo
        }
      }
    }
    // prefer our kernels unless another path is >5% faster
    route = 0;
    if (t[2] < 0.95f * t[route]) route = 2;
    if (t[3] < 0.95f * t[route]) route = 3;
    if (t[1] < 0.95f * t[route]) route = 1;
    std::lock_guard<std::mutex> g(g_route_mu);
    g_route[key] = route;
    g_route_ms[key] = t;
    g_p8_cfg[key] = p8c;
  }
  // a "lib" decision under policy 0 (or for an epilogue the library cannot
  // run): the fastest of our kernels the decision's timings recorded
  if (route == 1 && !lib_ok) {
    std::lock_guard<std::mutex> g(g_route_mu);
    const auto t = g_route_ms[key];
    route = 0;
    if (dma_ok && t[2] < t[route]) route = 2;
    auto pc = g_p8_cfg.find(key);
    if (p8_ok && pc != g_p8_cfg.end() && pc->second.first > 0 && t[3] < t[route]) route = 3;
  }
  std::pair<int, int> p8c{-1, -1};
  if (route == 3) {
    std::lock_guard<std::mutex> g(g_route_mu);
    auto it = g_p8_cfg.find(key);
    if (it != g_p8_cfg.end()) p8c = it->second;
  }
  if (route == 1) run_lib(a, a_kmajor, b, b_kmajor, c, mode, bias);
  else if (route == 3) run_p8(a, a_kmajor, b, b_kmajor, M, N, K, ep, allow_split, p8c.first, p8c.second);
  else run_mfma(a, a_kmajor, b, b_kmajor, M, N, K, ep, allow_split, route);
}

void gemm_lib_policy_op(int64_t p) { g_lib_policy = (int)p; }

// cached routing decisions: "M N K layout mode f32 epilogue route t_mfma t_lib t_dma (ms)" per line
std::string gemm_routes_op() {
  std::lock_guard<std::mutex> g(g_route_mu);
  std::ostringstream o;
  for (const auto& kv : g_route) {
    const auto& k = kv.first;
    const auto t = g_route_ms[k];
    o << std::get<0>(k) << " " << std::get<1>(k) << " " << std::get<2>(k) << " "
      << (std::get<3>(k) ? "K" : "M") << (std::get<4>(k) ? "K" : "N") << " " << std::get<5>(k)
      << " " << std::get<6>(k) << " " << std::get<7>(k) << " "
      << (kv.second == 1 ? "lib" : kv.second == 2 ? "dma" : kv.second == 3 ? "p8" : "mfma") << " " << t[0]
      << " " << t[1] << " " << t[2] << " " << t[3];
    auto pc = g_p8_cfg.find(k);
    if (pc != g_p8_cfg.end()) o << " " << pc->second.first << " " << pc->second.second;
    o << "\n";
  }
  return o.str();
}

// Pre-load routing decisions (the format gemm_routes() prints): a per-device
// tuning table shipped with the framework / saved by an earlier process, so
// a cold process does not time every GEMM shape on its jobs' first steps
// (like a library's tuned-solution database). Keys already decided in this
// process are kept. Returns the number of keys loaded.
int64_t gemm_routes_load_op(const std::string& text) {
  std::istringstream in(text);
  std::string line;
  int64_t n = 0;
  std::lock_guard<std::mutex> g(g_route_mu);
  while (std::getline(in, line)) {
    std::istringstream ls(line);
    int64_t M, N, K, mode;
    std::string lay, rt;
    int f32, epi;
    std::array<float, 4> t{};
    if (!(ls >> M >> N >> K >> lay >> mode >> f32 >> epi >> rt >> t[0] >> t[1] >> t[2] >> t[3])) continue;
    if (lay.size() != 2 || M <= 0 || N <= 0 || K <= 0) continue;
    const int route = rt == "lib" ? 1 : rt == "dma" ? 2 : rt == "p8" ? 3 : rt == "mfma" ? 0 : -1;
    if (route < 0) continue;
    const GemmKey key{M, N, K, lay[0] == 'K', lay[1] == 'K', mode, (bool)f32, (bool)epi};
    if (g_route.count(key)) continue;
    int tile = -1, sp = -1;
    const bool has_cfg = (bool)(ls >> tile >> sp);
    const bool cfg_ok = has_cfg &&
                        (tile == 128 || tile == 256 || ((tile == 64 || tile == 65 || tile == 129) && lay[0] == 'K')) &&
                        sp >= (tile == 256 ? 0 : 1) && sp <= 16;
    if (route == 3 && !cfg_ok) continue;                // a p8 route needs its measured config
    g_route[key] = route;
    g_route_ms[key] = t;
    // kept for any route: a "lib" decision falls back to the p8 config it
    // was timed against when the library is switched off
    if (cfg_ok) g_p8_cfg[key] = {tile, sp};
    ++n;
  }
  return n;
}

// ------------------------------------------------------------------ conv
tam::ConvGeom geom(const Tensor& x, const Tensor& w, const Tensor& y, int64_t stride, int64_t pad,
                   int64_t dil) {
  tam::ConvGeom g;
  g.N = (int)x.size(0); g.H = (int)x.size(1); g.W = (int)x.size(2); g.C = (int)x.size(3);
  g.K = (int)w.size(0); g.R = (int)w.size(1); g.S = (int)w.size(2);
  g.P = (int)y.size(1); g.Q = (int)y.size(2);
  g.stride = (int)stride; g.pad = (int)pad; g.dil = (int)dil;
  TORCH_CHECK(w.size(3) == g.C, "tam.conv: weight C mismatch");
  TORCH_CHECK(y.size(0) == g.N && y.size(3) == g.K, "tam.conv: output shape mismatch");
  TORCH_CHECK(g.P == (g.H + 2 * g.pad - g.dil * (g.R - 1) - 1) / g.stride + 1 &&
                  g.Q == (g.W + 2 * g.pad - g.dil * (g.S - 1) - 1) / g.stride + 1,
              "tam.conv: output spatial size inconsistent with geometry");
  TORCH_CHECK(g.C % 8 == 0 && g.K % 8 == 0, "tam.conv: C and K must be multiples of 8");
  return g;
}

// stats (optional, fp64 [2K], zeroed by the caller): BatchNorm sums of y
// accumulated by the conv epilogue; returns 1 when they were (0: this path
// computes none, the BN reduces y itself)
int64_t conv_fwd_op(const Tensor& x, const Tensor& w, const Tensor& y, int64_t stride, int64_t pad,
                    int64_t dil, const optional<Tensor>& bias, bool relu, const optional<Tensor>& stats) {
  check_bf16(x, "x"); check_bf16(w, "w"); check_bf16(y, "y");
  check_contig(x, "x"); check_contig(w, "w"); check_contig(y, "y");
  tam::ConvGeom g = geom(x, w, y, stride, pad, dil);
  tam::Epi ep;
  ep.c = y.data_ptr(); ep.ldc = g.K; ep.c_f32 = 0; ep.mode = 0;
  ep.bias = opt_ptr<const tam::bf16_t>(bias);
  ep.relu = relu;
  if (stats.has_value() && stats->defined()) {
    TORCH_CHECK(stats->is_cuda() && stats->scalar_type() == at::kDouble && stats->is_contiguous() &&
                stats->numel() == tam::BN_SHARDS * 2 * g.K,
                "tam.conv_fwd: stats must be a contiguous fp64 [BN_SHARDS * 2K] tensor");
    ep.stats = stats->data_ptr<double>();
  }
  const long wsf = tam::conv_fwd_split_ws(g);
  Tensor ws;
  if (wsf > 0) ws = at::empty({wsf}, x.options().dtype(at::kFloat));
  return tam::conv_fwd(bp(x), bp(w), g, ep, cur_stream(x), wsf > 0 ? ws.data_ptr<float>() : nullptr, wsf);
}

void conv_dgrad_op(const Tensor& dy, const Tensor& w, const Tensor& wt, const Tensor& dx,
                   int64_t stride, int64_t pad, int64_t dil, const optional<Tensor>& mask) {
  check_bf16(dy, "dy"); check_bf16(w, "w"); check_bf16(dx, "dx");
  check_contig(dy, "dy"); check_contig(w, "w"); check_contig(dx, "dx");
  tam::ConvGeom g = geom(dx, w, dy, stride, pad, dil);
  // wt = W re-laid [C][R][S][K] (the K-major B operand of dgrad; for 1x1
  // convs the LDS-DMA core reads it, the plain-GEMM fallback does not)
  check_bf16(wt, "wt");
  TORCH_CHECK(wt.numel() == w.numel(), "tam.conv_dgrad: wt workspace size");
  tam::conv_weight_t(bp(w), bpm(wt), g, cur_stream(dy));
  tam::Epi ep;
  ep.c = dx.data_ptr(); ep.ldc = g.C; ep.c_f32 = 0; ep.mode = 0;
  if (mask.has_value() && mask->defined()) {
    check_bf16(*mask, "mask");
    TORCH_CHECK(mask->numel() == dx.numel(), "tam.conv_dgrad: mask size");
    ep.mask = bp(*mask); ep.ldm = g.C;
  }
  const long wsf = tam::conv_dgrad_split_ws(g);
  Tensor ws;
  if (wsf > 0) ws = at::empty({wsf}, dy.options().dtype(at::kFloat));
  tam::conv_dgrad(bp(dy), bp(w), bp(wt), g, ep, cur_stream(dy), wsf > 0 ? ws.data_ptr<float>() : nullptr, wsf);
}

// deferred weight gradients of many Linear layers in one grouped launch:
// dw[i] (fp32 [M][N]) += dy[i]^T x[i] (dy [T][M], x [T][N] bf16), db[i] (fp32
// [M], or an empty tensor for none) += colsum(dy[i])
void gemm_wgrad_grouped_op(at::TensorList dy, at::TensorList x, at::TensorList dw, at::TensorList db,
                           at::OptionalIntArrayRef modes) {
  TORCH_CHECK(dy.size() == x.size() && dy.size() == dw.size() && dy.size() == db.size(),
              "tam.gemm_wgrad_grouped: list sizes differ");
  TORCH_CHECK(!modes.has_value() || modes->size() == dy.size(), "tam.gemm_wgrad_grouped: modes size");
  if (dy.empty()) return;
  std::vector<tam::GGProblem> probs(dy.size());
  for (size_t i = 0; i < dy.size(); ++i) {
    const Tensor& a = dy[i];
    const Tensor& b = x[i];
    const Tensor& c = dw[i];
    check_bf16(a, "dy"); check_bf16(b, "x"); check_f32(c, "dw");
    check_contig(a, "dy"); check_contig(b, "x"); check_contig(c, "dw");
    TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2 && a.size(0) == b.size(0) &&
                    c.size(0) == a.size(1) && c.size(1) == b.size(1),
                "tam.gemm_wgrad_grouped: shapes dy [T,M], x [T,N], dw [M,N] expected");
    TORCH_CHECK(a.device() == dy[0].device() && b.device() == a.device() && c.device() == a.device(),
                "tam.gemm_wgrad_grouped: all operands on one device");
    const int M = (int)a.size(1), N = (int)b.size(1), K = (int)a.size(0);
    TORCH_CHECK(tam::gemm_wgrad_grouped_ok(M, N, K, M, N),
                "tam.gemm_wgrad_grouped: problem ", i, " (", M, "x", N, "x", K,
                ") not eligible (K % 64, M/N >= 128 and % 8)");
    float* bias = nullptr;
    if (db[i].defined() && db[i].numel() > 0) {
      check_f32(db[i], "db");
      TORCH_CHECK(db[i].numel() == M && db[i].is_contiguous(), "tam.gemm_wgrad_grouped: db must be [M]");
      bias = db[i].data_ptr<float>();
    }
    const int mode = modes.has_value() ? (int)(*modes)[i] : 1;
    TORCH_CHECK(mode == 0 || mode == 1, "tam.gemm_wgrad_grouped: mode must be 0 (store) or 1 (accumulate)");
    probs[i] = tam::GGProblem{bp(a), bp(b), c.data_ptr<float>(), bias, M, N, K, M, N, mode};
  }
  tam::gemm_wgrad_grouped(probs.data(), (int)probs.size(), cur_stream(dy[0]));
}

void gemm_grouped_tile_op(int64_t t) { tam::gemm_grouped_tile((int)t); }

bool gemm_wgrad_grouped_ok_op(int64_t M, int64_t N, int64_t K) {
  return tam::gemm_wgrad_grouped_ok((int)M, (int)N, (int)K, M, N);
}

// every conv weight of a model re-laid for dgrad in one launch
void conv_weight_t_batch_op(at::TensorList w, at::TensorList wt) {
  TORCH_CHECK(w.size() == wt.size(), "tam.conv_weight_t_batch: list sizes differ");
  if (w.empty()) return;
  hipStream_t st = cur_stream(w[0]);
  for (size_t base = 0; base < w.size(); base += tam::WT_MAX) {
    tam::WTBatch b{};
    b.n = (int)std::min<size_t>(tam::WT_MAX, w.size() - base);
    for (int i = 0; i < b.n; ++i) {
      const Tensor& a = w[base + i];
      const Tensor& t = wt[base + i];
      check_bf16(a, "w"); check_bf16(t, "wt"); check_contig(a, "w"); check_contig(t, "wt");
      TORCH_CHECK(a.dim() == 4 && t.numel() == a.numel(), "tam.conv_weight_t_batch: w must be [K,R,S,C]");
      b.e[i].w = bp(a); b.e[i].wt = bpm(t);
      b.e[i].K = (int)a.size(0); b.e[i].RS = (int)(a.size(1) * a.size(2)); b.e[i].C = (int)a.size(3);
    }
    tam::conv_weight_t_batch(b, st);
  }
}

// dgrad with wt already re-laid (conv_weight_t_batch)
// stats / bnx / bnmean / bnrstd (all or none): dx is the gradient of a
// BatchNorm output whose input was bnx; the dgrad epilogue then accumulates
// the BN-backward sums into stats (fp64 [2C], zeroed by the caller) and the
// op returns 1 (0: this shape's dgrad path computes none)
int64_t conv_dgrad_pre_op(const Tensor& dy, const Tensor& w, const Tensor& wt, const Tensor& dx,
                          int64_t stride, int64_t pad, int64_t dil, const optional<Tensor>& mask,
                          const optional<Tensor>& stats, const optional<Tensor>& bnx,
                          const optional<Tensor>& bnmean, const optional<Tensor>& bnrstd) {
  check_bf16(dy, "dy"); check_bf16(w, "w"); check_bf16(dx, "dx"); check_bf16(wt, "wt");
  check_contig(dy, "dy"); check_contig(w, "w"); check_contig(dx, "dx"); check_contig(wt, "wt");
  TORCH_CHECK(wt.numel() == w.numel(), "tam.conv_dgrad_pre: wt size");
  tam::ConvGeom g = geom(dx, w, dy, stride, pad, dil);
  tam::Epi ep;
  ep.c = dx.data_ptr(); ep.ldc = g.C; ep.c_f32 = 0; ep.mode = 0;
  if (mask.has_value() && mask->defined()) {
    check_bf16(*mask, "mask");
    TORCH_CHECK(mask->numel() == dx.numel(), "tam.conv_dgrad_pre: mask size");
    ep.mask = bp(*mask); ep.ldm = g.C;
  }
  if (stats.has_value() && stats->defined()) {
    TORCH_CHECK(bnx.has_value() && bnmean.has_value() && bnrstd.has_value(),
                "tam.conv_dgrad_pre: stats needs bnx, bnmean, bnrstd");
    check_bf16(*bnx, "bnx"); check_f32(*bnmean, "bnmean"); check_f32(*bnrstd, "bnrstd");
    check_contig(*bnx, "bnx");
    TORCH_CHECK(stats->is_cuda() && stats->scalar_type() == at::kDouble && stats->is_contiguous() &&
                stats->numel() == tam::BN_SHARDS * 2 * g.C && bnx->numel() == dx.numel() && bnmean->numel() == g.C &&
                bnrstd->numel() == g.C, "tam.conv_dgrad_pre: BN-backward operand shapes");
    ep.stats = stats->data_ptr<double>();
    ep.bnx = bp(*bnx);
    ep.bnmean = bnmean->data_ptr<float>();
    ep.bnrstd = bnrstd->data_ptr<float>();
  }
  const long wsf = ep.bnx ? 0 : tam::conv_dgrad_split_ws(g);
  Tensor ws;
  if (wsf > 0) ws = at::empty({wsf}, dy.options().dtype(at::kFloat));
  return tam::conv_dgrad(bp(dy), bp(w), bp(wt), g, ep, cur_stream(dy), wsf > 0 ? ws.data_ptr<float>() : nullptr,
                         wsf);
}

// dbias (optional, fp32 [K]): += the bias gradient colsum(dY), fused into the
// wgrad kernel where it has the epilogue, else a column-sum pass
// conv_wgrad_deferred: as conv_wgrad, but a slab-split pass leaves its
// reduce to the caller: returns (slabs, sp) -- sp > 0: dw is NOT written yet;
// wgrad_slab_reduce_many([slabs], [sp], [dw], [mode]) finishes it (batched
// over a backward). sp == 0: dw is complete (slabs is empty)
std::tuple<Tensor, int64_t> conv_wgrad_deferred_op(const Tensor& dy, const Tensor& x, const Tensor& dw,
                                                   int64_t stride, int64_t pad, int64_t dil, int64_t mode,
                                                   const optional<Tensor>& dbias, bool patch) {
  check_bf16(dy, "dy"); check_bf16(x, "x"); check_f32(dw, "dw");
  check_contig(dy, "dy"); check_contig(x, "x"); check_contig(dw, "dw");
  TORCH_CHECK(dw.dim() == 4, "tam.conv_wgrad_deferred: dw must be [K,R,S,C]");
  tam::ConvGeom g = geom(x, dw, dy, stride, pad, dil);
  tam::Epi ep;
  ep.c = dw.data_ptr(); ep.ldc = g.R * g.S * g.C; ep.c_f32 = 1; ep.mode = (int)mode;
  float* db = nullptr;
  if (dbias.has_value() && dbias->defined()) {
    check_f32(*dbias, "dbias");
    TORCH_CHECK(dbias->numel() == g.K && dbias->is_contiguous(), "tam.conv_wgrad_deferred: dbias size");
    db = dbias->data_ptr<float>();
  }
  const long wsf = tam::conv_wgrad_split_ws(g);
  Tensor wsl = at::empty({wsf > 0 ? wsf : 0}, dy.options().dtype(at::kFloat));
  int sp = 0;
  const int fused = tam::conv_wgrad(bp(dy), bp(x), g, ep, cur_stream(dy), db, patch,
                                    wsf > 0 ? wsl.data_ptr<float>() : nullptr, wsf, &sp);
  if (db && !fused) {
    const long R = (long)g.N * g.P * g.Q;
    Tensor ws = at::empty({g.K % 8 == 0 ? (int64_t)tam::COLSUM_MAX_BLOCKS * g.K : 1}, dy.options().dtype(at::kFloat));
    tam::colsum(bp(dy), db, ws.data_ptr<float>(), R, g.K, cur_stream(dy));
  }
  return {sp > 0 ? wsl : at::empty({0}, dy.options().dtype(at::kFloat)), (int64_t)sp};
}

void wgrad_slab_reduce_many_op(at::TensorList slabs, at::IntArrayRef sp, at::TensorList dw, at::IntArrayRef mode) {
  const size_t n = slabs.size();
  TORCH_CHECK(sp.size() == n && dw.size() == n && mode.size() == n, "tam.wgrad_slab_reduce_many: list sizes");
  if (n == 0) return;
  std::vector<const float*> ws(n);
  std::vector<float*> out(n);
  std::vector<int> s(n), md(n);
  std::vector<long> mn(n);
  for (size_t i = 0; i < n; ++i) {
    check_f32(slabs[i], "slab"); check_f32(dw[i], "dw");
    TORCH_CHECK(dw[i].is_contiguous() && dw[i].numel() % 4 == 0 && sp[i] > 0 &&
                    slabs[i].numel() >= sp[i] * dw[i].numel(),
                "tam.wgrad_slab_reduce_many: entry ", i);
    ws[i] = slabs[i].data_ptr<float>();
    out[i] = dw[i].data_ptr<float>();
    s[i] = (int)sp[i];
    md[i] = (int)mode[i];
    mn[i] = (long)dw[i].numel();
  }
  tam::wgrad_slab_reduce_many(ws.data(), s.data(), mn.data(), out.data(), md.data(), (int)n, cur_stream(dw[0]));
}

void conv_wgrad_op(const Tensor& dy, const Tensor& x, const Tensor& dw, int64_t stride, int64_t pad,
                   int64_t dil, int64_t mode, const optional<Tensor>& dbias, bool patch) {
  check_bf16(dy, "dy"); check_bf16(x, "x"); check_f32(dw, "dw");
  check_contig(dy, "dy"); check_contig(x, "x"); check_contig(dw, "dw");
  TORCH_CHECK(dw.dim() == 4, "tam.conv_wgrad: dw must be [K,R,S,C]");
  tam::ConvGeom g = geom(x, dw, dy, stride, pad, dil);
  tam::Epi ep;
  ep.c = dw.data_ptr(); ep.ldc = g.R * g.S * g.C; ep.c_f32 = 1; ep.mode = (int)mode;
  float* db = nullptr;
  if (dbias.has_value() && dbias->defined()) {
    check_f32(*dbias, "dbias");
    TORCH_CHECK(dbias->numel() == g.K && dbias->is_contiguous(), "tam.conv_wgrad: dbias size");
    db = dbias->data_ptr<float>();
  }
  const long wsf = tam::conv_wgrad_split_ws(g);
  Tensor wsl;
  if (wsf > 0) wsl = at::empty({wsf}, dy.options().dtype(at::kFloat));
  const int fused = tam::conv_wgrad(bp(dy), bp(x), g, ep, cur_stream(dy), db, patch,
                                    wsf > 0 ? wsl.data_ptr<float>() : nullptr, wsf);
  if (db && !fused) {
    const long R = (long)g.N * g.P * g.Q;
    Tensor ws = at::empty({g.K % 8 == 0 ? (int64_t)tam::COLSUM_MAX_BLOCKS * g.K : 1}, dy.options().dtype(at::kFloat));
    tam::colsum(bp(dy), db, ws.data_ptr<float>(), R, g.K, cur_stream(dy));
  }
}

// ------------------------------------------------------------------ norms
// sums (optional): fp64 [BN_SHARDS][2C] BN statistics workspace. sums_ready:
// already accumulated (the producing conv's epilogue); otherwise it must be
// zeroed and the reduction pass stores into it. Absent: a zeroed temporary.
static double* bn_sums(const optional<Tensor>& sums, const Tensor& x, int64_t C, Tensor& tmp,
                       const char* what) {
  if (sums.has_value() && sums->defined()) {
    TORCH_CHECK(sums->is_cuda() && sums->scalar_type() == at::kDouble && sums->is_contiguous() &&
                sums->numel() == tam::BN_SHARDS * 2 * C, what,
                ": sums must be a contiguous fp64 [BN_SHARDS * 2C] tensor");
    return sums->data_ptr<double>();
  }
  tmp = at::zeros({tam::BN_SHARDS * 2 * C}, x.options().dtype(at::kDouble));
  return tmp.data_ptr<double>();
}

void bn_forward_op(const Tensor& x, const optional<Tensor>& res, const Tensor& y, const Tensor& gamma,
                   const Tensor& beta, const optional<Tensor>& run_mean,
                   const optional<Tensor>& run_var, const Tensor& save_mean,
                   const Tensor& save_rstd, double eps, double momentum, bool relu,
                   const optional<Tensor>& sums, bool sums_ready, const optional<Tensor>& ymask) {
  check_bf16(x, "x"); check_bf16(y, "y"); check_contig(x, "x"); check_contig(y, "y");
  check_f32(gamma, "gamma"); check_f32(beta, "beta");
  const int64_t C = x.size(-1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "tam.bn: C must be a multiple of 8 and <= 2048");
  TORCH_CHECK(!sums_ready || (sums.has_value() && sums->defined()), "tam.bn_forward: sums_ready without sums");
  if (res.has_value() && res->defined()) { check_bf16(*res, "res"); check_contig(*res, "res"); }
  Tensor tmp;
  double* sp = bn_sums(sums, x, C, tmp, "tam.bn_forward");
  uint8_t* mp = nullptr;
  if (ymask.has_value() && ymask->defined()) {
    TORCH_CHECK(relu && ymask->is_cuda() && ymask->scalar_type() == at::kByte && ymask->is_contiguous() &&
                ymask->numel() == x.numel() / 8, "tam.bn_forward: ymask must be uint8 [numel/8] (relu only)");
    mp = ymask->data_ptr<uint8_t>();
  }
  tam::bn_forward(bp(x), opt_ptr<const tam::bf16_t>(res), bpm(y), M, (int)C, (float)eps,
                  (float)momentum, gamma.data_ptr<float>(), beta.data_ptr<float>(),
                  opt_ptr<float>(run_mean), opt_ptr<float>(run_var), save_mean.data_ptr<float>(),
                  save_rstd.data_ptr<float>(), relu, sp, sums_ready ? 1 : 0, mp, cur_stream(x));
}

void bn_backward_op(const Tensor& dy, const optional<Tensor>& y, const Tensor& x, const Tensor& mean,
                    const Tensor& rstd, const Tensor& gamma, const Tensor& dx,
                    const optional<Tensor>& dres, const optional<Tensor>& dgamma,
                    const optional<Tensor>& dbeta, bool relu, const optional<Tensor>& addend,
                    const optional<Tensor>& sums, bool sums_ready, const optional<Tensor>& ymask) {
  check_bf16(dy, "dy"); check_bf16(x, "x"); check_bf16(dx, "dx");
  check_contig(dy, "dy"); check_contig(x, "x"); check_contig(dx, "dx");
  const int64_t C = x.size(-1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "tam.bn: C must be a multiple of 8 and <= 2048");
  const bool has_mask = ymask.has_value() && ymask->defined();
  TORCH_CHECK(!relu || (y.has_value() && y->defined()) || has_mask, "tam.bn_backward: relu needs y or ymask");
  if (has_mask)
    TORCH_CHECK(ymask->is_cuda() && ymask->scalar_type() == at::kByte && ymask->is_contiguous() &&
                ymask->numel() == x.numel() / 8, "tam.bn_backward: ymask must be uint8 [numel/8]");
  const tam::bf16_t* yp = has_mask ? nullptr : opt_ptr<const tam::bf16_t>(y);
  const bool has_add = addend.has_value() && addend->defined();
  if (has_add) {
    check_bf16(*addend, "addend"); check_contig(*addend, "addend");
    TORCH_CHECK(addend->numel() == dy.numel(), "tam.bn_backward: addend size");
  }
  TORCH_CHECK(!sums_ready || ((sums.has_value() && sums->defined()) && !relu && !has_add &&
                              !(dres.has_value() && dres->defined())),
              "tam.bn_backward: sums_ready takes the already-masked gradient (no relu / addend / dres)");
  Tensor tmp;
  double* sp = bn_sums(sums, x, C, tmp, "tam.bn_backward");
  tam::bn_backward(bp(dy), opt_ptr<const tam::bf16_t>(addend), yp, bp(x), mean.data_ptr<float>(),
                   rstd.data_ptr<float>(), gamma.data_ptr<float>(), M, (int)C, relu, bpm(dx),
                   opt_ptr<tam::bf16_t>(dres), opt_ptr<float>(dgamma), opt_ptr<float>(dbeta),
                   sp, sums_ready ? 1 : 0, has_mask ? ymask->data_ptr<uint8_t>() : nullptr, cur_stream(x));
}

// addend / sum_out (both or neither): y = LN(x + addend), sum_out = x + addend
void ln_forward_op(const Tensor& x, const Tensor& g, const Tensor& b, const Tensor& y,
                   const Tensor& mean, const Tensor& rstd, double eps, const optional<Tensor>& addend,
                   const optional<Tensor>& sum_out) {
  check_bf16(x, "x"); check_bf16(y, "y"); check_contig(x, "x"); check_contig(y, "y");
  check_f32(g, "g"); check_f32(b, "b");
  const int64_t D = x.size(-1);
  TORCH_CHECK(D % 8 == 0 && D <= 2048, "tam.ln: D must be a multiple of 8 and <= 2048");
  const bool add = addend.has_value() && addend->defined();
  TORCH_CHECK(add == (sum_out.has_value() && sum_out->defined()), "tam.ln_forward: addend needs sum_out");
  if (add) {
    check_bf16(*addend, "addend"); check_contig(*addend, "addend");
    check_bf16(*sum_out, "sum_out"); check_contig(*sum_out, "sum_out");
    TORCH_CHECK(addend->numel() == x.numel() && sum_out->numel() == x.numel(), "tam.ln_forward: addend size");
  }
  tam::ln_forward(bp(x), g.data_ptr<float>(), b.data_ptr<float>(), bpm(y), mean.data_ptr<float>(),
                  rstd.data_ptr<float>(), x.numel() / D, (int)D, (float)eps, cur_stream(x),
                  add ? bp(*addend) : nullptr, add ? bpm(*sum_out) : nullptr);
}

void ln_backward_op(const Tensor& dy, const Tensor& x, const Tensor& g, const Tensor& mean,
                    const Tensor& rstd, const Tensor& dx, const Tensor& dg, const Tensor& db,
                    const optional<Tensor>& addend) {
  check_bf16(dy, "dy"); check_bf16(x, "x"); check_bf16(dx, "dx");
  check_contig(dy, "dy"); check_contig(x, "x"); check_contig(dx, "dx");
  check_f32(dg, "dg"); check_f32(db, "db");
  const tam::bf16_t* add = nullptr;
  if (addend.has_value() && addend->defined()) {
    check_bf16(*addend, "addend"); check_contig(*addend, "addend");
    TORCH_CHECK(addend->numel() == x.numel(), "tam.ln_backward: addend size");
    add = bp(*addend);
  }
  const int64_t D = x.size(-1);
  Tensor ws = at::empty({(int64_t)tam::LN_MAX_BLOCKS * 2 * D}, x.options().dtype(at::kFloat));
  tam::ln_backward(bp(dy), bp(x), g.data_ptr<float>(), mean.data_ptr<float>(),
                   rstd.data_ptr<float>(), bpm(dx), add, dg.data_ptr<float>(), db.data_ptr<float>(),
                   ws.data_ptr<float>(), x.numel() / D, (int)D, cur_stream(x));
}

// LN backward without its column reduce: per-block partials into ws (fp32,
// >= LN_MAX_BLOCKS * 2D); returns the partial-row count for col_reduce_acc
int64_t ln_backward_split_op(const Tensor& dy, const Tensor& x, const Tensor& g, const Tensor& mean,
                             const Tensor& rstd, const Tensor& dx, const Tensor& ws,
                             const optional<Tensor>& addend) {
  check_bf16(dy, "dy"); check_bf16(x, "x"); check_bf16(dx, "dx");
  check_contig(dy, "dy"); check_contig(x, "x"); check_contig(dx, "dx");
  check_f32(ws, "ws");
  const int64_t D = x.size(-1);
  TORCH_CHECK(ws.is_contiguous() && ws.numel() >= (int64_t)tam::LN_MAX_BLOCKS * 2 * D,
              "tam.ln_backward_split: ws must hold LN_MAX_BLOCKS * 2D floats");
  const tam::bf16_t* add = nullptr;
  if (addend.has_value() && addend->defined()) {
    check_bf16(*addend, "addend"); check_contig(*addend, "addend");
    TORCH_CHECK(addend->numel() == x.numel(), "tam.ln_backward_split: addend size");
    add = bp(*addend);
  }
  return tam::ln_backward_partial(bp(dy), bp(x), g.data_ptr<float>(), mean.data_ptr<float>(),
                                  rstd.data_ptr<float>(), bpm(dx), add, ws.data_ptr<float>(), x.numel() / D,
                                  (int)D, cur_stream(x));
}

// out0[c] += sum_b part[b][c] (c < split), out1[c - split] += ... (c >= split)
void col_reduce_acc_op(const Tensor& part, int64_t nblk, int64_t W, const Tensor& out0, const Tensor& out1,
                       int64_t split) {
  check_f32(part, "part"); check_f32(out0, "out0"); check_f32(out1, "out1");
  TORCH_CHECK(part.is_contiguous() && part.numel() >= nblk * W && out0.numel() == split &&
                  out1.numel() == W - split && out0.is_contiguous() && out1.is_contiguous(),
              "tam.col_reduce_acc: shapes");
  tam::col_reduce_acc(part.data_ptr<float>(), (int)nblk, (int)W, out0.data_ptr<float>(), out1.data_ptr<float>(),
                      (int)split, cur_stream(part));
}

// many col_reduce_acc in one launch: parts[i] [nblk[i]][W[i]] fp32 partial
// rows; out0[i][c] += sum (c < split[i]), out1[i][c - split[i]] += sum
void col_reduce_acc_batch_op(at::TensorList parts, at::IntArrayRef nblk, at::TensorList out0,
                             at::TensorList out1) {
  const size_t n = parts.size();
  TORCH_CHECK(nblk.size() == n && out0.size() == n && out1.size() == n, "tam.col_reduce_acc_batch: list sizes");
  if (n == 0) return;
  std::vector<const float*> pp(n);
  std::vector<float*> o0(n), o1(n);
  std::vector<int> nb(n), W(n), sp(n);
  for (size_t i = 0; i < n; ++i) {
    check_f32(parts[i], "part"); check_f32(out0[i], "out0"); check_f32(out1[i], "out1");
    sp[i] = (int)out0[i].numel();
    W[i] = sp[i] + (int)out1[i].numel();
    nb[i] = (int)nblk[i];
    TORCH_CHECK(parts[i].is_contiguous() && parts[i].numel() >= (int64_t)nb[i] * W[i] &&
                    out0[i].is_contiguous() && out1[i].is_contiguous() && parts[i].device() == parts[0].device(),
                "tam.col_reduce_acc_batch: entry ", i);
    pp[i] = parts[i].data_ptr<float>();
    o0[i] = out0[i].data_ptr<float>();
    o1[i] = out1[i].data_ptr<float>();
  }
  tam::col_reduce_acc_batch(pp.data(), nb.data(), W.data(), o0.data(), o1.data(), sp.data(), (int)n,
                            cur_stream(parts[0]));
}

// ------------------------------------------------------------------ pooling
void maxpool_forward_op(const Tensor& x, const Tensor& y, const Tensor& idx, int64_t R, int64_t S,
                        int64_t st, int64_t pad) {
  check_bf16(x, "x"); check_bf16(y, "y"); check_contig(x, "x"); check_contig(y, "y");
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.numel() == y.numel(), "tam.maxpool: idx");
  tam::maxpool_forward(bp(x), bpm(y), idx.data_ptr<uint8_t>(), (int)x.size(0), (int)x.size(1),
                       (int)x.size(2), (int)x.size(3), (int)y.size(1), (int)y.size(2), (int)R,
                       (int)S, (int)st, (int)pad, cur_stream(x));
}
void maxpool_k3s2_policy_op(int64_t p) { tam::maxpool_k3s2_policy((int)p); }
void maxpool_backward_op(const Tensor& dy, const Tensor& idx, const Tensor& dx, int64_t R, int64_t S,
                         int64_t st, int64_t pad) {
  check_bf16(dy, "dy"); check_bf16(dx, "dx");
  tam::maxpool_backward(bp(dy), idx.data_ptr<uint8_t>(), bpm(dx), (int)dx.size(0), (int)dx.size(1),
                        (int)dx.size(2), (int)dx.size(3), (int)dy.size(1), (int)dy.size(2), (int)R,
                        (int)S, (int)st, (int)pad, cur_stream(dy));
}
void avgpool_forward_op(const Tensor& x, const Tensor& y) {
  check_bf16(x, "x"); check_bf16(y, "y"); check_contig(x, "x");
  tam::avgpool_forward(bp(x), bpm(y), (int)x.size(0), (int)(x.size(1) * x.size(2)), (int)x.size(3),
                       cur_stream(x));
}
void avgpool_backward_op(const Tensor& dy, const Tensor& dx) {
  check_bf16(dy, "dy"); check_bf16(dx, "dx"); check_contig(dx, "dx");
  tam::avgpool_backward(bp(dy), bpm(dx), (int)dx.size(0), (int)(dx.size(1) * dx.size(2)),
                        (int)dx.size(3), cur_stream(dy));
}

// ------------------------------------------------------------------ loss / embed / misc
void softmax_xent_op(const Tensor& logits, const Tensor& labels, const optional<Tensor>& dlogits,
                     const Tensor& loss_rows, double smoothing, double grad_scale,
                     int64_t ignore_index, int64_t tm_b) {
  check_bf16(logits, "logits"); check_contig(logits, "logits");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_cuda() && labels.is_contiguous(),
              "tam.xent: labels contiguous int64 GPU");
  check_f32(loss_rows, "loss_rows");
  const int64_t V = logits.size(-1), rows = logits.numel() / V;
  TORCH_CHECK(labels.numel() == rows && loss_rows.numel() == rows, "tam.xent: row count");
  TORCH_CHECK(tm_b <= 0 || rows % tm_b == 0, "tam.xent: tm_b must divide the rows");
  tam::softmax_xent(bp(logits), labels.data_ptr<int64_t>(), opt_ptr<tam::bf16_t>(dlogits),
                    loss_rows.data_ptr<float>(), rows, (int)V, (float)smoothing, (float)grad_scale,
                    ignore_index, cur_stream(logits), tm_b);
}

void embedding_forward_op(const Tensor& table, const Tensor& ids, const Tensor& out, double scale, int64_t tm_b,
                          const optional<Tensor>& pos) {
  check_bf16(table, "table"); check_bf16(out, "out"); check_contig(table, "table");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous(), "tam.embedding: ids");
  const int64_t D = table.size(1);
  TORCH_CHECK(D % 8 == 0, "tam.embedding: D % 8");
  TORCH_CHECK(out.numel() == ids.numel() * D, "tam.embedding: out size");
  TORCH_CHECK(tm_b <= 0 || ids.numel() % tm_b == 0, "tam.embedding: tm_b must divide the ids");
  const tam::bf16_t* pp = nullptr;
  int64_t prow = 0;
  if (pos.has_value() && pos->defined()) {
    check_bf16(*pos, "pos"); check_contig(*pos, "pos");
    TORCH_CHECK(pos->dim() == 2 && pos->size(1) == D, "tam.embedding: pos must be [S][D]");
    prow = pos->size(0);
    TORCH_CHECK(prow > 0 && (tm_b > 0 ? ids.numel() / tm_b == prow : ids.numel() % prow == 0),
                "tam.embedding: pos rows must equal the sequence length");
    pp = bp(*pos);
  }
  tam::embedding_forward(bp(table), ids.data_ptr<int64_t>(), bpm(out), ids.numel(), (int)D,
                         (float)scale, cur_stream(table), table.size(0), tm_b, pp, prow);
}
void embedding_backward_op(const Tensor& dout, const Tensor& ids, const Tensor& gtable, double scale, int64_t tm_b) {
  check_bf16(dout, "dout"); check_f32(gtable, "gtable"); check_contig(dout, "dout");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous() && gtable.dim() == 2 &&
                  dout.numel() == ids.numel() * gtable.size(1), "tam.embedding_backward: shapes");
  TORCH_CHECK(tm_b <= 0 || ids.numel() % tm_b == 0, "tam.embedding_backward: tm_b must divide the ids");
  tam::embedding_backward(bp(dout), ids.data_ptr<int64_t>(), gtable.data_ptr<float>(), ids.numel(),
                          (int)gtable.size(1), (float)scale, cur_stream(dout), gtable.size(0), tm_b);
}

void conv_dma_policy_op(int64_t p) { tam::conv_dma_policy((int)p); }
void conv_halo_policy_op(int64_t p) { tam::conv_halo_policy((int)p); }
void colsum_policy_op(int64_t p) { tam::colsum_policy((int)p); }
void attn_short_policy_op(int64_t p) { tam::attn_short_policy((int)p); }
// forced (bm, bn, splits) of the LDS-DMA conv wgrad (A/B sweeps; 0 = heuristic)
void conv_wgrad_c64_policy_op(int64_t p) { tam::conv_wgrad_c64_policy((int)p); }
void conv_wgrad_order_op(int64_t p) { tam::conv_wgrad_order((int)p); }
void conv_stem_policy_op(int64_t p) { tam::conv_stem_policy((int)p); }
void conv_wgrad_slab_policy_op(int64_t p) { tam::conv_wgrad_slab_policy((int)p); }
void conv_wgrad_force_op(int64_t bm, int64_t bn, int64_t splits, int64_t noatomic) {
  tam::conv_wgrad_force((int)bm, (int)bn, (int)splits, (int)noatomic);
}
// 0: never the LDS-DMA GEMM; 1: measured per-shape routing (default);
// 2: LDS-DMA GEMM wherever eligible, tile cfg forced when >= 0 (tests/sweeps)
int g_dma_policy = 1;
TAM_KNOB(g_dma_policy)
void gemm_dma_policy_op(int64_t p, int64_t cfg) {
  g_dma_policy = (int)p;
  tam::gemm_dma_policy(p == 2 ? 1 : 0, (int)cfg);
}

void gemm8p_policy_op(int64_t mode, int64_t tile) { tam::gemm8p_policy((int)mode, (int)tile); }
void gemm_pw_policy_op(int64_t on) { tam::gemm_pw_policy((int)on); }

// every registered tuning knob (common.h TAM_KNOB): names (comma-joined, in
// registration order), current values, and a bulk restore
std::string policy_names_op() {
  std::string out;
  for (const auto& k : tam::knob_registry()) {
    if (!out.empty()) out += ",";
    out += k.name;
  }
  return out;
}
std::vector<int64_t> policy_state_op() {
  std::vector<int64_t> v;
  for (const auto& k : tam::knob_registry()) v.push_back(*k.p);
  return v;
}
void policy_load_op(std::vector<int64_t> v) {
  auto& reg = tam::knob_registry();
  TORCH_CHECK(v.size() == reg.size(), "policy_load: ", v.size(), " values for ", reg.size(), " knobs");
  for (size_t i = 0; i < reg.size(); ++i) *reg[i].p = (int)v[i];
}
void gemm8p_group_op(int64_t g) { tam::gemm8p_group((int)g); }
void gemm8p_slab_force_op(int64_t sp) { tam::gemm8p_slab_force((int)sp); }
void gemm8p_sk_force_op(int64_t on) { g_sk_force = on != 0; }
void conv_split_policy_op(int64_t p) { tam::conv_split_policy((int)p); }
void optim_grid_op(int64_t b) { tam::optim_grid((int)b); }
void optim_variant_op(int64_t v) { tam::optim_variant((int)v); }
void gemm_skinny_policy_op(int64_t on, int64_t sp, int64_t nst) {
  tam::gemm_skinny_policy((int)on, (int)sp, (int)nst);
}
// C[M][N] = A[M][K] . B[N][K]^T through the 4-wave 256^2 kernel (A/B and tests)

void gemm_force_op(int64_t cfg, int64_t splits) {
  tam::gemm_force((int)cfg, (int)splits);
  g_forced = cfg >= 0 || splits >= 1;
}

void colsum_op(const Tensor& x, const Tensor& out) {
  check_bf16(x, "x"); check_f32(out, "out"); check_contig(x, "x");
  const int64_t C = x.size(-1);
  Tensor ws = at::empty({C % 8 == 0 ? (int64_t)tam::COLSUM_MAX_BLOCKS * C : 1},
                        x.options().dtype(at::kFloat));
  tam::colsum(bp(x), out.data_ptr<float>(), ws.data_ptr<float>(), x.numel() / C, (int)C,
              cur_stream(x));
}
void relu_backward_op(const Tensor& dy, const Tensor& y, const Tensor& dx) {
  check_bf16(dy, "dy"); check_bf16(y, "y"); check_bf16(dx, "dx");
  tam::relu_backward(bp(dy), bp(y), bpm(dx), dy.numel(), cur_stream(dy));
}
void sum_scale_op(const Tensor& x, const Tensor& out, double scale) {
  check_f32(x, "x"); check_f32(out, "out"); check_contig(x, "x");
  TORCH_CHECK(out.numel() >= 1, "tam.sum_scale: out");
  tam::sum_scale(x.data_ptr<float>(), x.numel(), out.data_ptr<float>(), (float)scale, cur_stream(x));
}
// a 2-D row view of a bf16 [..., C] tensor whose leading dims collapse to
// rows at one pitch (a last-dim slice of a contiguous tensor qualifies)
static std::pair<int64_t, int64_t> row_view(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() >= 1 && t.stride(-1) == 1,
              "tam.rows_sum: ", what, " must be a bf16 CUDA tensor with unit last stride");
  const int64_t C = t.size(-1);
  int64_t ld = t.dim() >= 2 ? t.stride(-2) : C;
  for (int64_t d = t.dim() - 2; d >= 1; --d)
    TORCH_CHECK(t.size(d) == 1 || t.size(d - 1) == 1 || t.stride(d - 1) == t.stride(d) * t.size(d),
                "tam.rows_sum: ", what, " leading dims do not collapse to one row pitch");
  TORCH_CHECK(C % 8 == 0 && ld % 8 == 0 && (((uintptr_t)t.data_ptr()) & 15) == 0,
              "tam.rows_sum: ", what, " needs C % 8 == 0 and 16-B aligned rows");
  return {C, ld};
}
// outs[j] = sum of the next n_in[j] tensors of ins (row-pitched views, one row count)
void rows_sum_op(at::TensorList outs, at::TensorList ins, at::IntArrayRef n_in) {
  TORCH_CHECK(!outs.empty() && outs.size() <= 4 && outs.size() == n_in.size(), "tam.rows_sum: 1-4 jobs");
  const int64_t R = outs[0].numel() / outs[0].size(-1);
  tam::RowJobs jb{};
  size_t q = 0;
  for (size_t j = 0; j < outs.size(); ++j) {
    auto [C, ld] = row_view(outs[j], "out");
    TORCH_CHECK(outs[j].numel() / C == R, "tam.rows_sum: every job needs the same row count");
    TORCH_CHECK(n_in[j] >= 1 && n_in[j] <= 4 && q + n_in[j] <= ins.size(), "tam.rows_sum: n_in");
    tam::RowJob& r = jb.job[j];
    r.out = bpm(outs[j]); r.ld_out = ld; r.C = (int)C; r.n_in = (int)n_in[j];
    for (int k = 0; k < r.n_in; ++k, ++q) {
      auto [Ci, ldi] = row_view(ins[q], "in");
      TORCH_CHECK(Ci == C && ins[q].numel() / Ci == R, "tam.rows_sum: input shape");
      r.in[k] = bp(ins[q]); r.ld_in[k] = ldi;
    }
  }
  TORCH_CHECK(q == ins.size(), "tam.rows_sum: unused inputs");
  tam::rows_sum(jb, (int)outs.size(), R, cur_stream(outs[0]));
}
void zero_op(const Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "tam.zero_: contiguous CUDA tensor");
  tam::zero_async(t.data_ptr(), t.numel() * t.element_size(), cur_stream(t));
}
void add_op(const Tensor& a, const Tensor& b, const Tensor& y) {
  check_bf16(a, "a"); check_bf16(b, "b"); check_bf16(y, "y");
  TORCH_CHECK(a.numel() % 8 == 0, "tam.add: numel % 8");
  tam::add_bf16(bp(a), bp(b), bpm(y), a.numel(), cur_stream(a));
}
void cast_op(const Tensor& x, const Tensor& y) {
  check_f32(x, "x"); check_bf16(y, "y");
  tam::cast_f32_bf16(x.data_ptr<float>(), bpm(y), x.numel(), cur_stream(x));
}

// ------------------------------------------------------------------ optimizers
// guard (optional int32 [2], the job's persistent-LSTM error words): a
// non-zero guard[0] turns the step into a gradient reset (optim.hip)
static const unsigned* guard_ptr(const optional<Tensor>& guard, const Tensor& like) {
  if (!(guard.has_value() && guard->defined())) return nullptr;
  TORCH_CHECK(guard->scalar_type() == at::kInt && guard->numel() >= 2 && guard->device() == like.device(),
              "tam: guard must be an int32 [2] tensor on the parameters' device");
  return (const unsigned*)guard->data_ptr<int>();
}
void sgd_op(const Tensor& w, const Tensor& g, const Tensor& mom, const Tensor& wb, double lr,
            double momentum, double wd, double gscale, bool nesterov, bool zero_grad,
            const optional<Tensor>& guard, int64_t zero_from, int64_t wd_until) {
  check_f32(w, "w"); check_f32(g, "g"); check_f32(mom, "mom"); check_bf16(wb, "wb");
  TORCH_CHECK(w.numel() % 4 == 0 && g.numel() == w.numel() && mom.numel() == w.numel() &&
                  wb.numel() == w.numel(),
              "tam.sgd: sizes");
  TORCH_CHECK(zero_from % 4 == 0 && (wd_until < 0 || wd_until % 4 == 0), "tam.sgd: region bounds % 4");
  tam::sgd_step(w.data_ptr<float>(), g.data_ptr<float>(), mom.data_ptr<float>(), bpm(wb), w.numel(),
                (float)lr, (float)momentum, (float)wd, (float)gscale, nesterov, zero_grad,
                cur_stream(w), guard_ptr(guard, w), (long)zero_from, (long)wd_until);
}
void adam_op(const Tensor& w, const Tensor& g, const Tensor& m, const Tensor& v, const Tensor& wb,
             double lr, double b1, double b2, double eps, double wd, int64_t step, double gscale,
             bool zero_grad, const optional<Tensor>& guard, int64_t zero_from, int64_t wd_until) {
  check_f32(w, "w"); check_f32(g, "g"); check_f32(m, "m"); check_f32(v, "v"); check_bf16(wb, "wb");
  TORCH_CHECK(w.numel() % 4 == 0, "tam.adam: numel % 4");
  TORCH_CHECK(zero_from % 4 == 0 && (wd_until < 0 || wd_until % 4 == 0), "tam.adam: region bounds % 4");
  tam::adam_step(w.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                 bpm(wb), w.numel(), (float)lr, (float)b1, (float)b2, (float)eps, (float)wd,
                 (int)step, (float)gscale, zero_grad, cur_stream(w), guard_ptr(guard, w), (long)zero_from,
                 (long)wd_until);
}
void lstm_guard_step_op(const Tensor& err) {
  TORCH_CHECK(err.is_cuda() && err.scalar_type() == at::kInt && err.numel() >= 2,
              "tam.lstm_guard_step: err must be an int32 [2] GPU tensor");
  tam::lstm_guard_step((unsigned*)err.data_ptr<int>(), cur_stream(err));
}

// ------------------------------------------------------------------ attention
// q,k,v,o: [B,S,H,64] views (unit stride on d, stride 64 on heads)
void check_attn_view(const Tensor& t, const char* name) {
  check_bf16(t, name);
  TORCH_CHECK(t.dim() == 4 && t.size(3) == 64 && t.stride(3) == 1 && t.stride(2) == 64,
              "tam.attn: ", name, " must be a [B,S,H,64] view with packed heads");
  // any batch / token strides (batch-major [B,S,.] or a time-major [S,B,.]
  // tensor viewed transposed), 16-byte aligned rows
  TORCH_CHECK(t.stride(1) % 8 == 0 && t.stride(0) % 8 == 0, "tam.attn: ", name, " stride alignment");
}
void attn_forward_op(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o,
                     const Tensor& lse, bool causal, double scale, const optional<Tensor>& kv_len) {
  check_attn_view(q, "q"); check_attn_view(k, "k"); check_attn_view(v, "v"); check_attn_view(o, "o");
  TORCH_CHECK(k.stride(1) == v.stride(1), "tam.attn: k/v token strides differ");
  check_f32(lse, "lse");
  const int B = (int)q.size(0), Sq = (int)q.size(1), H = (int)q.size(2), Sk = (int)k.size(1);
  TORCH_CHECK(lse.numel() == (int64_t)B * H * Sq, "tam.attn: lse size");
  TORCH_CHECK(k.stride(0) == v.stride(0), "tam.attn: k/v batch strides differ");
  tam::attn_forward(bp(q), bp(k), bp(v), bpm(o), lse.data_ptr<float>(), B, H, Sq, Sk, q.stride(1),
                    k.stride(1), o.stride(1), q.stride(0), k.stride(0), o.stride(0), causal, (float)scale,
                    opt_ptr<const int>(kv_len), cur_stream(q));
}
void attn_backward_op(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o,
                      const Tensor& dout, const Tensor& lse, const Tensor& dq, const Tensor& dk,
                      const Tensor& dv, const Tensor& dq_acc, const Tensor& delta, bool causal,
                      double scale, const optional<Tensor>& kv_len) {
  check_attn_view(q, "q"); check_attn_view(k, "k"); check_attn_view(v, "v"); check_attn_view(o, "o");
  check_attn_view(dout, "dout"); check_attn_view(dq, "dq"); check_attn_view(dk, "dk");
  check_attn_view(dv, "dv");
  TORCH_CHECK(dout.stride(1) == o.stride(1) && dout.stride(0) == o.stride(0), "tam.attn_bwd: dout must match o layout");
  TORCH_CHECK(dq.stride(1) == q.stride(1) && dk.stride(1) == k.stride(1) && dv.stride(1) == k.stride(1) &&
                  dq.stride(0) == q.stride(0) && dk.stride(0) == k.stride(0) && dv.stride(0) == k.stride(0) &&
                  v.stride(0) == k.stride(0) && v.stride(1) == k.stride(1),
              "tam.attn_bwd: grads must match input layouts");
  const int B = (int)q.size(0), Sq = (int)q.size(1), H = (int)q.size(2), Sk = (int)k.size(1);
  check_f32(dq_acc, "dq_acc"); check_f32(delta, "delta");
  TORCH_CHECK(dq_acc.numel() >= (int64_t)B * Sq * H * 64 && delta.numel() >= (int64_t)B * H * Sq,
              "tam.attn_bwd: workspace sizes");
  tam::attn_backward(bp(q), bp(k), bp(v), bp(o), bp(dout), lse.data_ptr<float>(), bpm(dq), bpm(dk),
                     bpm(dv), dq_acc.data_ptr<float>(), delta.data_ptr<float>(), B, H, Sq, Sk,
                     q.stride(1), k.stride(1), o.stride(1), q.stride(0), k.stride(0), o.stride(0), causal,
                     (float)scale,
                     opt_ptr<const int>(kv_len), cur_stream(q));
}

// ------------------------------------------------------------------ LSTM
void lstm_fwd_op(const Tensor& gates, const optional<Tensor>& c_prev, const Tensor& c_out,
                 const Tensor& h_out, const optional<Tensor>& h_f32, const Tensor& act) {
  check_f32(gates, "gates"); check_f32(c_out, "c_out"); check_bf16(h_out, "h_out"); check_f32(act, "act");
  const int B = (int)gates.size(0), Hd = (int)(gates.size(1) / 4);
  tam::lstm_cell_forward(gates.data_ptr<float>(), opt_ptr<const float>(c_prev), c_out.data_ptr<float>(),
                         bpm(h_out), opt_ptr<float>(h_f32), act.data_ptr<float>(), B, Hd,
                         cur_stream(gates));
}
// fused timestep: gx [B][4Hd] f32 (x-projection + bias), w_hh [4Hd][Hd] bf16
void lstm_step_fwd_op(const Tensor& gx, const Tensor& w_hh, const optional<Tensor>& h_prev,
                      const optional<Tensor>& c_prev, const Tensor& c_out, const Tensor& h_out,
                      const Tensor& act) {
  check_f32(gx, "gx"); check_bf16(w_hh, "w_hh"); check_f32(c_out, "c_out"); check_bf16(h_out, "h_out");
  check_f32(act, "act");
  const int64_t B = gx.size(0), Hd = w_hh.size(1);
  TORCH_CHECK(gx.dim() == 2 && gx.size(1) == 4 * Hd && gx.stride(1) == 1 && gx.stride(0) == 4 * Hd,
              "tam.lstm_step_forward: gx must be contiguous [B][4*Hd]");
  TORCH_CHECK(w_hh.is_contiguous() && w_hh.size(0) == 4 * Hd, "tam.lstm_step_forward: w_hh [4Hd][Hd]");
  TORCH_CHECK(B % 16 == 0 && Hd % 256 == 0, "tam.lstm_step_forward: needs B % 16 == 0, Hd % 256 == 0");
  TORCH_CHECK(c_out.numel() == B * Hd && h_out.numel() == B * Hd && act.numel() == 5 * B * Hd &&
              c_out.is_contiguous() && h_out.is_contiguous() && act.is_contiguous(),
              "tam.lstm_step_forward: output shapes");
  if (h_prev.has_value() && h_prev->defined()) {
    check_bf16(*h_prev, "h_prev");
    TORCH_CHECK(h_prev->is_contiguous() && h_prev->numel() == B * Hd, "tam.lstm_step_forward: h_prev");
  }
  if (c_prev.has_value() && c_prev->defined()) {
    check_f32(*c_prev, "c_prev");
    TORCH_CHECK(c_prev->is_contiguous() && c_prev->numel() == B * Hd, "tam.lstm_step_forward: c_prev");
  }
  tam::lstm_step_forward(gx.data_ptr<float>(), bp(w_hh), opt_ptr<const tam::bf16_t>(h_prev),
                         opt_ptr<const float>(c_prev), c_out.data_ptr<float>(), bpm(h_out),
                         act.data_ptr<float>(), (int)B, (int)Hd, cur_stream(gx));
}

// persistent whole-sequence recurrence; returns false when the shape or
// co-residency is not supported (caller runs the per-step path).
// sync: int32 [32 * (4 * B/16 + 1)] = {error flag, up to 4 arrival counters
// per batch tile on lines of their own} -- all zeroed by the launcher (the
// caller may pass uninitialised memory)
static void check_sync(const Tensor& sync, int64_t B) {
  TORCH_CHECK(sync.is_cuda() && sync.scalar_type() == at::kInt && sync.is_contiguous() &&
              sync.numel() >= 32 * (4 * (B / 16) + 1),
              "tam.lstm_seq: sync must be a contiguous int32 tensor of >= 32 * (4 * B/16 + 1) elements");
}
// per-launch co-residency rule + the job's timeout word (see tam::PLOpts)
static tam::PLOpts pl_opts(const optional<Tensor>& job_err, int64_t grids, int64_t rsv, bool zeroed) {
  tam::PLOpts o;
  o.grids = (int)grids;
  o.rsv = (int)rsv;
  o.zeroed = zeroed ? 1 : 0;
  if (job_err.has_value() && job_err->defined()) {
    TORCH_CHECK(job_err->is_cuda() && job_err->scalar_type() == at::kInt && job_err->numel() >= 2,
                "tam.lstm_seq: job_err must be an int32 [2] GPU tensor");
    o.job_err = (unsigned*)job_err->data_ptr<int>();
  }
  return o;
}
bool lstm_seq_fwd_op(const Tensor& gx, const Tensor& w_hh, const Tensor& hs, const Tensor& cs,
                     const Tensor& act, bool reverse, const Tensor& sync, const optional<Tensor>& job_err,
                     int64_t grids, int64_t rsv, bool zeroed) {
  check_f32(gx, "gx"); check_bf16(w_hh, "w_hh"); check_bf16(hs, "hs"); check_f32(cs, "cs");
  check_f32(act, "act");
  TORCH_CHECK(hs.dim() == 3 && hs.is_contiguous(), "tam.lstm_seq_forward: hs [T][B][Hd]");
  const int64_t T = hs.size(0), B = hs.size(1), Hd = hs.size(2);
  check_sync(sync, B);
  TORCH_CHECK(w_hh.is_contiguous() && w_hh.size(0) == 4 * Hd && w_hh.size(1) == Hd,
              "tam.lstm_seq_forward: w_hh [4Hd][Hd]");
  TORCH_CHECK(gx.is_contiguous() && gx.numel() == T * B * 4 * Hd, "tam.lstm_seq_forward: gx [T][B][4Hd]");
  TORCH_CHECK(cs.is_contiguous() && cs.numel() == T * B * Hd && act.is_contiguous() &&
              act.numel() == T * B * 5 * Hd, "tam.lstm_seq_forward: cs / act shapes");
  int* sp = sync.data_ptr<int>();
  return tam::lstm_seq_forward(gx.data_ptr<float>(), bp(w_hh), bpm(hs), cs.data_ptr<float>(),
                               act.data_ptr<float>(), (int)T, (int)B, (int)Hd, reverse ? 1 : 0,
                               (unsigned*)sp, cur_stream(gx), pl_opts(job_err, grids, rsv, zeroed));
}
bool lstm_seq_bwd_op(const Tensor& act, const Tensor& cs, const Tensor& dH, const Tensor& w_hh,
                     const Tensor& dG, bool reverse, const Tensor& sync, const optional<Tensor>& job_err,
                     int64_t grids, int64_t rsv, bool zeroed) {
  check_f32(act, "act"); check_f32(cs, "cs"); check_bf16(w_hh, "w_hh");
  TORCH_CHECK(dH.is_cuda() && (dH.scalar_type() == at::kFloat || dH.scalar_type() == at::kBFloat16),
              "tam.lstm_seq_backward: dH must be an f32 or bf16 CUDA tensor");
  const int dh_bf16 = dH.scalar_type() == at::kBFloat16 ? 1 : 0;
  check_bf16(dG, "dG");
  TORCH_CHECK(cs.dim() == 3 && cs.is_contiguous(), "tam.lstm_seq_backward: cs [T][B][Hd]");
  const int64_t T = cs.size(0), B = cs.size(1), Hd = cs.size(2);
  check_sync(sync, B);
  TORCH_CHECK(w_hh.is_contiguous() && w_hh.size(0) == 4 * Hd && w_hh.size(1) == Hd,
              "tam.lstm_seq_backward: w_hh [4Hd][Hd]");
  // dH: contiguous [T][B][Hd], or a [T][B][Hd] column slice of a wider row
  // (row pitch ldh = stride(1), stride(0) = B * ldh): read in place
  TORCH_CHECK(dH.dim() == 3 && dH.size(0) == T && dH.size(1) == B && dH.size(2) == Hd && dH.stride(2) == 1 &&
                  dH.stride(1) >= Hd && dH.stride(0) == B * dH.stride(1),
              "tam.lstm_seq_backward: dH [T][B][Hd] with unit column stride and uniform row pitch");
  TORCH_CHECK(act.is_contiguous() && act.numel() == T * B * 5 * Hd && dG.is_contiguous() &&
                  dG.numel() == T * B * 4 * Hd,
              "tam.lstm_seq_backward: act / dG shapes");
  int* sp = sync.data_ptr<int>();
  return tam::lstm_seq_backward(act.data_ptr<float>(), cs.data_ptr<float>(), (const float*)dH.data_ptr(),
                                bp(w_hh), bpm(dG), (int)T, (int)B, (int)Hd, reverse ? 1 : 0, (unsigned*)sp,
                                dh_bf16, (int)dH.stride(1), cur_stream(act), pl_opts(job_err, grids, rsv, zeroed));
}

void lstm_seq_policy_op(int64_t ch) { tam::lstm_seq_policy((int)ch); }
void lstm_seq_shards_op(int64_t ns) { tam::lstm_seq_shards((int)ns); }
void lstm_seq_residency_op(int64_t grids, int64_t rsv) { tam::lstm_seq_residency((int)grids, (int)rsv); }
int64_t lstm_persist_timeouts_op(bool reset) { return tam::lstm_persist_timeouts(reset); }
void lstm_seq_spin_limit_op(int64_t polls) { tam::lstm_seq_spin_limit(polls); }

void lstm_bwd_op(const Tensor& act, const optional<Tensor>& c_prev, const optional<Tensor>& dh,
                 const optional<Tensor>& dc_next, const optional<Tensor>& dgates,
                 const optional<Tensor>& dc_prev, const optional<Tensor>& dgates_bf16) {
  check_f32(act, "act");
  const int B = (int)act.size(0), Hd = (int)(act.size(1) / 5);
  tam::lstm_cell_backward(act.data_ptr<float>(), opt_ptr<const float>(c_prev), nullptr,
                          opt_ptr<const float>(dh), opt_ptr<const float>(dc_next),
                          opt_ptr<float>(dgates), opt_ptr<float>(dc_prev),
                          opt_ptr<tam::bf16_t>(dgates_bf16), B, Hd, c10::hip::getCurrentHIPStream(act.device().index()).stream());
}

}  // namespace

TORCH_LIBRARY(tam, m) {
  m.def("gemm(Tensor a, bool a_kmajor, Tensor b, bool b_kmajor, Tensor(a!) c, int mode, Tensor? bias, bool relu, Tensor? mask, float alpha, bool allow_split, Tensor(b!)? colsum=None) -> ()", &gemm_op);
  m.def("conv_fwd(Tensor x, Tensor w, Tensor(a!) y, int stride, int pad, int dil, Tensor? bias, bool relu, Tensor(b!)? stats=None) -> int", &conv_fwd_op);
  m.def("conv_dgrad(Tensor dy, Tensor w, Tensor(a!) wt, Tensor(b!) dx, int stride, int pad, int dil, Tensor? mask) -> ()", &conv_dgrad_op);
  m.def("conv_weight_t_batch(Tensor[] w, Tensor(a!)[] wt) -> ()", &conv_weight_t_batch_op);
  m.def("gemm_wgrad_grouped(Tensor[] dy, Tensor[] x, Tensor(a!)[] dw, Tensor(b!)[] db, int[]? modes=None) -> ()", &gemm_wgrad_grouped_op);
  m.def("gemm_wgrad_grouped_ok(int M, int N, int K) -> bool", &gemm_wgrad_grouped_ok_op);
  m.def("gemm_grouped_tile(int tile) -> ()", &gemm_grouped_tile_op);
  m.def("conv_dgrad_pre(Tensor dy, Tensor w, Tensor wt, Tensor(a!) dx, int stride, int pad, int dil, Tensor? mask, Tensor(b!)? stats=None, Tensor? bnx=None, Tensor? bnmean=None, Tensor? bnrstd=None) -> int", &conv_dgrad_pre_op);
  m.def("conv_wgrad(Tensor dy, Tensor x, Tensor(a!) dw, int stride, int pad, int dil, int mode, Tensor(b!)? dbias=None, bool patch=True) -> ()", &conv_wgrad_op);
  m.def("conv_wgrad_deferred(Tensor dy, Tensor x, Tensor(a!) dw, int stride, int pad, int dil, int mode, Tensor(b!)? dbias, bool patch) -> (Tensor, int)", &conv_wgrad_deferred_op);
  m.def("wgrad_slab_reduce_many(Tensor[] slabs, int[] sp, Tensor(a!)[] dw, int[] mode) -> ()", &wgrad_slab_reduce_many_op);
  m.def("bn_forward(Tensor x, Tensor? res, Tensor(a!) y, Tensor gamma, Tensor beta, Tensor(b!)? run_mean, Tensor(c!)? run_var, Tensor(d!) save_mean, Tensor(e!) save_rstd, float eps, float momentum, bool relu, Tensor(f!)? sums=None, bool sums_ready=False, Tensor(g!)? ymask=None) -> ()", &bn_forward_op);
  m.def("bn_backward(Tensor dy, Tensor? y, Tensor x, Tensor mean, Tensor rstd, Tensor gamma, Tensor(a!) dx, Tensor(b!)? dres, Tensor(c!)? dgamma, Tensor(d!)? dbeta, bool relu, Tensor? addend=None, Tensor(e!)? sums=None, bool sums_ready=False, Tensor? ymask=None) -> ()", &bn_backward_op);
  m.def("ln_forward(Tensor x, Tensor g, Tensor b, Tensor(a!) y, Tensor(b!) mean, Tensor(c!) rstd, float eps, Tensor? addend=None, Tensor(d!)? sum_out=None) -> ()", &ln_forward_op);
  m.def("ln_backward(Tensor dy, Tensor x, Tensor g, Tensor mean, Tensor rstd, Tensor(a!) dx, Tensor(b!) dg, Tensor(c!) db, Tensor? addend=None) -> ()", &ln_backward_op);
  m.def("ln_backward_split(Tensor dy, Tensor x, Tensor g, Tensor mean, Tensor rstd, Tensor(a!) dx, Tensor(b!) ws, Tensor? addend=None) -> int", &ln_backward_split_op);
  m.def("col_reduce_acc(Tensor part, int nblk, int W, Tensor(a!) out0, Tensor(b!) out1, int split) -> ()", &col_reduce_acc_op);
  m.def("col_reduce_acc_batch(Tensor[] parts, int[] nblk, Tensor(a!)[] out0, Tensor(b!)[] out1) -> ()", &col_reduce_acc_batch_op);
  m.def("maxpool_forward(Tensor x, Tensor(a!) y, Tensor(b!) idx, int R, int S, int stride, int pad) -> ()", &maxpool_forward_op);
  m.def("maxpool_backward(Tensor dy, Tensor idx, Tensor(a!) dx, int R, int S, int stride, int pad) -> ()", &maxpool_backward_op);
  m.def("maxpool_k3s2_policy(int policy) -> ()", &maxpool_k3s2_policy_op);
  m.def("avgpool_forward(Tensor x, Tensor(a!) y) -> ()", &avgpool_forward_op);
  m.def("avgpool_backward(Tensor dy, Tensor(a!) dx) -> ()", &avgpool_backward_op);
  m.def("softmax_xent(Tensor logits, Tensor labels, Tensor(a!)? dlogits, Tensor(b!) loss_rows, float smoothing, float grad_scale, int ignore_index, int tm_b=0) -> ()", &softmax_xent_op);
  m.def("embedding_forward(Tensor table, Tensor ids, Tensor(a!) out, float scale, int tm_b=0, Tensor? pos=None) -> ()", &embedding_forward_op);
  m.def("embedding_backward(Tensor dout, Tensor ids, Tensor(a!) gtable, float scale, int tm_b=0) -> ()", &embedding_backward_op);
  m.def("sum_scale(Tensor x, Tensor(a!) out, float scale) -> ()", &sum_scale_op);
  m.def("rows_sum(Tensor[] outs, Tensor[] ins, int[] n_in) -> ()", &rows_sum_op);
  m.def("zero_(Tensor(a!) t) -> ()", &zero_op);
  m.def("colsum(Tensor x, Tensor(a!) out) -> ()", &colsum_op);
  m.def("gemm_force(int cfg, int splits) -> ()", &gemm_force_op);
  m.def("gemm8p_policy(int mode, int tile) -> ()", &gemm8p_policy_op);
  m.def("gemm_pw_policy(int on) -> ()", &gemm_pw_policy_op);
  m.def("policy_names() -> str", &policy_names_op);
  m.def("policy_state() -> int[]", &policy_state_op);
  m.def("policy_load(int[] v) -> ()", &policy_load_op);
  m.def("gemm8p_group(int g) -> ()", &gemm8p_group_op);
  m.def("gemm8p_slab_force(int sp) -> ()", &gemm8p_slab_force_op);
  m.def("gemm_skinny_policy(int on, int force_splits, int nst) -> ()", &gemm_skinny_policy_op);
  m.def("gemm8p_sk_force(int on) -> ()", &gemm8p_sk_force_op);
  m.def("conv_split_policy(int p) -> ()", &conv_split_policy_op);
  m.def("optim_variant(int v) -> ()", &optim_variant_op);
  m.def("optim_grid(int blocks) -> ()", &optim_grid_op);
  m.def("gemm_lib_policy(int policy) -> ()", &gemm_lib_policy_op);
  m.def("conv_dma_policy(int policy) -> ()", &conv_dma_policy_op);
  m.def("conv_wgrad_force(int bm, int bn, int splits, int noatomic=0) -> ()", &conv_wgrad_force_op);
  m.def("conv_wgrad_c64_policy(int policy) -> ()", &conv_wgrad_c64_policy_op);
  m.def("conv_wgrad_order(int flat) -> ()", &conv_wgrad_order_op);
  m.def("conv_stem_policy(int policy) -> ()", &conv_stem_policy_op);
  m.def("conv_wgrad_slab_policy(int policy) -> ()", &conv_wgrad_slab_policy_op);
  m.def("conv_halo_policy(int policy) -> ()", &conv_halo_policy_op);
  m.def("colsum_policy(int policy) -> ()", &colsum_policy_op);
  m.def("attn_short_policy(int policy) -> ()", &attn_short_policy_op);
  m.def("gemm_dma_policy(int policy, int cfg) -> ()", &gemm_dma_policy_op);
  m.def("gemm_routes() -> str", &gemm_routes_op);
  m.def("relu_backward(Tensor dy, Tensor y, Tensor(a!) dx) -> ()", &relu_backward_op);
  m.def("add(Tensor a, Tensor b, Tensor(a!) y) -> ()", &add_op);
  m.def("cast_f32_bf16(Tensor x, Tensor(a!) y) -> ()", &cast_op);
  m.def("sgd_step(Tensor(a!) w, Tensor(b!) g, Tensor(c!) mom, Tensor(d!) wb, float lr, float momentum, float wd, float gscale, bool nesterov, bool zero_grad, Tensor? guard=None, int zero_from=0, int wd_until=-1) -> ()", &sgd_op);
  m.def("adam_step(Tensor(a!) w, Tensor(b!) g, Tensor(c!) m, Tensor(d!) v, Tensor(e!) wb, float lr, float b1, float b2, float eps, float wd, int step, float gscale, bool zero_grad, Tensor? guard=None, int zero_from=0, int wd_until=-1) -> ()", &adam_op);
  m.def("lstm_guard_step(Tensor(a!) err) -> ()", &lstm_guard_step_op);
  m.def("attn_forward(Tensor q, Tensor k, Tensor v, Tensor(a!) o, Tensor(b!) lse, bool causal, float scale, Tensor? kv_len) -> ()", &attn_forward_op);
  m.def("attn_backward(Tensor q, Tensor k, Tensor v, Tensor o, Tensor dout, Tensor lse, Tensor(a!) dq, Tensor(b!) dk, Tensor(c!) dv, Tensor(d!) dq_acc, Tensor(e!) delta, bool causal, float scale, Tensor? kv_len) -> ()", &attn_backward_op);
  m.def("lstm_step_forward(Tensor gx, Tensor w_hh, Tensor? h_prev, Tensor? c_prev, Tensor(a!) c_out, Tensor(b!) h_out, Tensor(c!) act) -> ()", &lstm_step_fwd_op);
  m.def("lstm_seq_forward(Tensor gx, Tensor w_hh, Tensor(a!) hs, Tensor(b!) cs, Tensor(c!) act, bool reverse, Tensor(d!) sync, Tensor(e!)? job_err=None, int grids=-1, int reserved_cus=0, bool zeroed=False) -> bool", &lstm_seq_fwd_op);
  m.def("lstm_seq_backward(Tensor act, Tensor cs, Tensor dH, Tensor w_hh, Tensor(a!) dG, bool reverse, Tensor(b!) sync, Tensor(c!)? job_err=None, int grids=-1, int reserved_cus=0, bool zeroed=False) -> bool", &lstm_seq_bwd_op);
  m.def("lstm_seq_policy(int ch) -> ()", &lstm_seq_policy_op);
  m.def("lstm_seq_shards(int ns) -> ()", &lstm_seq_shards_op);
  m.def("gemm_routes_load(str text) -> int", &gemm_routes_load_op);
  m.def("lstm_seq_residency(int grids, int reserved_cus) -> ()", &lstm_seq_residency_op);
  m.def("lstm_persist_timeouts(bool reset) -> int", &lstm_persist_timeouts_op);
  m.def("lstm_seq_spin_limit(int polls) -> ()", &lstm_seq_spin_limit_op);
  m.def("lstm_cell_forward(Tensor gates, Tensor? c_prev, Tensor(a!) c_out, Tensor(b!) h_out, Tensor(c!)? h_f32, Tensor(d!) act) -> ()", &lstm_fwd_op);
  m.def("lstm_cell_backward(Tensor act, Tensor? c_prev, Tensor? dh, Tensor? dc_next, Tensor(a!)? dgates, Tensor(b!)? dc_prev, Tensor(c!)? dgates_bf16) -> ()", &lstm_bwd_op);
}
