// tiresias_amd — checkpoint spill/restore engine for preempted jobs.
//
// A preempted job's state (flat fp32 master params + optimizer state) stays
// resident in HBM while memory allows ("suspend in place": resume is a
// pointer swap). When the scheduler needs the HBM, the state is spilled to a
// pinned host pool with hipMemcpyAsync on a dedicated LOW-priority side
// stream, ordered after the producer stream by an event, so the spill
// overlaps the next job's compute. Restore is the reverse (H2D on the side
// stream; the consumer stream waits on an event, never the host).
//
// The pinned pool (tam/pinned_pool.h, host-only and sanitizer-tested) is
// carved from large hipHostMalloc'd chunks with a first-fit free list
// (coalescing on free) so spills never call the (synchronising, expensive)
// pinned allocator on the hot path.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <chrono>
#include <map>
#include <mutex>
#include <vector>

#include "tam/common.h"
#include "tam/pinned_pool.h"

namespace {

void* pinned_alloc(size_t n) {
  void* p = nullptr;
  TAM_HIP_CHECK(hipHostMalloc(&p, n, hipHostMallocDefault));
  return p;
}
void pinned_free(void* p) { (void)hipHostFree(p); }
using PinnedPool = tam::PinnedPool<void* (*)(size_t), void (*)(void*)>;

struct Spill {
  char* host = nullptr;
  size_t bytes = 0;
  hipEvent_t start = nullptr;   // D2H timing events on the side stream
  hipEvent_t done = nullptr;
  hipEvent_t rstart = nullptr;  // H2D (restore) timing events, created on the first restore
  hipEvent_t rdone = nullptr;
  std::vector<int64_t> shape;
  at::ScalarType dtype;
};

class CkptEngine : public torch::CustomClassHolder {
 public:
  CkptEngine(int64_t device, int64_t chunk_bytes)
      : device_((int)device), pool_((size_t)chunk_bytes, pinned_alloc, pinned_free) {
    TAM_HIP_CHECK(hipSetDevice(device_));
    int lo = 0, hi = 0;
    TAM_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    // numerically larger value = lower priority on HIP
    TAM_HIP_CHECK(hipStreamCreateWithPriority(&side_, hipStreamNonBlocking, lo));
  }
  ~CkptEngine() override {
    for (auto& kv : spills_) {
      if (kv.second.done) (void)hipEventDestroy(kv.second.done);
      if (kv.second.start) (void)hipEventDestroy(kv.second.start);
      if (kv.second.rstart) (void)hipEventDestroy(kv.second.rstart);
      if (kv.second.rdone) (void)hipEventDestroy(kv.second.rdone);
    }
    (void)hipStreamDestroy(side_);
  }

  // Asynchronously copy `src` (GPU) to pinned host memory. Ordered after all
  // work already queued on the caller's current stream.
  int64_t spill(const at::Tensor& src) {
    TORCH_CHECK(src.is_cuda() && src.is_contiguous(), "ckpt.spill: contiguous GPU tensor required");
    std::lock_guard<std::mutex> g(mu_);
    Spill s;
    s.bytes = src.numel() * src.element_size();
    s.host = pool_.alloc(s.bytes);
    s.shape = src.sizes().vec();
    s.dtype = src.scalar_type();
    hipStream_t prod = c10::hip::getCurrentHIPStream(src.device().index()).stream();
    hipEvent_t ready;
    TAM_HIP_CHECK(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    TAM_HIP_CHECK(hipEventRecord(ready, prod));
    TAM_HIP_CHECK(hipStreamWaitEvent(side_, ready, 0));
    TAM_HIP_CHECK(hipEventCreate(&s.start));
    TAM_HIP_CHECK(hipEventRecord(s.start, side_));
    TAM_HIP_CHECK(hipMemcpyAsync(s.host, src.data_ptr(), s.bytes, hipMemcpyDeviceToHost, side_));
    TAM_HIP_CHECK(hipEventCreate(&s.done));
    TAM_HIP_CHECK(hipEventRecord(s.done, side_));
    TAM_HIP_CHECK(hipEventDestroy(ready));
    const int64_t h = next_++;
    spills_[h] = s;
    bytes_d2h_ += s.bytes;
    return h;
  }

  // Restore a spill into `dst` (GPU, same byte size). The caller's current
  // stream waits (device-side) for the copy; the host never blocks.
  void restore(int64_t h, const at::Tensor& dst) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = spills_.find(h);
    TORCH_CHECK(it != spills_.end(), "ckpt.restore: unknown handle ", h);
    Spill& s = it->second;
    TORCH_CHECK(dst.is_cuda() && dst.is_contiguous() &&
                    (size_t)(dst.numel() * dst.element_size()) == s.bytes,
                "ckpt.restore: destination size mismatch");
    hipStream_t cons = c10::hip::getCurrentHIPStream(dst.device().index()).stream();
    // the destination may still be in use by earlier work on the consumer stream
    hipEvent_t free_ev;
    TAM_HIP_CHECK(hipEventCreateWithFlags(&free_ev, hipEventDisableTiming));
    TAM_HIP_CHECK(hipEventRecord(free_ev, cons));
    TAM_HIP_CHECK(hipStreamWaitEvent(side_, free_ev, 0));
    TAM_HIP_CHECK(hipStreamWaitEvent(side_, s.done, 0));
    if (!s.rstart) TAM_HIP_CHECK(hipEventCreate(&s.rstart));
    if (!s.rdone) TAM_HIP_CHECK(hipEventCreate(&s.rdone));
    TAM_HIP_CHECK(hipEventRecord(s.rstart, side_));
    TAM_HIP_CHECK(hipMemcpyAsync(dst.data_ptr(), s.host, s.bytes, hipMemcpyHostToDevice, side_));
    TAM_HIP_CHECK(hipEventRecord(s.rdone, side_));
    TAM_HIP_CHECK(hipStreamWaitEvent(cons, s.rdone, 0));
    TAM_HIP_CHECK(hipEventDestroy(free_ev));
    bytes_h2d_ += s.bytes;
  }

  bool ready(int64_t h) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = spills_.find(h);
    TORCH_CHECK(it != spills_.end(), "ckpt.ready: unknown handle");
    return hipEventQuery(it->second.done) == hipSuccess;
  }

  void wait(int64_t h) {
    hipEvent_t e;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = spills_.find(h);
      TORCH_CHECK(it != spills_.end(), "ckpt.wait: unknown handle");
      e = it->second.done;
    }
    TAM_HIP_CHECK(hipEventSynchronize(e));
  }

  // Device time of the last copy of this spill (D2H, or the H2D after a
  // restore), ms; -1 while it is still in flight. Never blocks.
  // kind 0: the D2H spill, 1: the latest H2D restore (-2 if never restored)
  double copy_ms(int64_t h, int64_t kind) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = spills_.find(h);
    TORCH_CHECK(it != spills_.end(), "ckpt.copy_ms: unknown handle");
    hipEvent_t a = kind ? it->second.rstart : it->second.start;
    hipEvent_t b = kind ? it->second.rdone : it->second.done;
    if (!a || !b) return -2.0;
    if (hipEventQuery(b) != hipSuccess) return -1.0;
    float ms = 0.f;
    TAM_HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    return ms;
  }

  // The side stream's handle: Python wraps it (torch.cuda.ExternalStream)
  // to record_stream() a spilled buffer before freeing it, so the caching
  // allocator defers reusing that HBM until the D2H has drained — the host
  // never waits for a spill.
  int64_t stream_handle() { return (int64_t)(uintptr_t)side_; }

  // Free the host copy (after restore completes or when the job finished).
  void release(int64_t h) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = spills_.find(h);
    if (it == spills_.end()) return;
    TAM_HIP_CHECK(hipEventSynchronize(it->second.rdone ? it->second.rdone : it->second.done));
    TAM_HIP_CHECK(hipEventDestroy(it->second.done));
    TAM_HIP_CHECK(hipEventDestroy(it->second.start));
    if (it->second.rstart) TAM_HIP_CHECK(hipEventDestroy(it->second.rstart));
    if (it->second.rdone) TAM_HIP_CHECK(hipEventDestroy(it->second.rdone));
    pool_.free(it->second.host, it->second.bytes);
    spills_.erase(it);
  }

  // Host-side view of a spill (for tests / persisting to disk): a CPU tensor
  // aliasing the pinned buffer. Waits for the D2H to complete.
  at::Tensor host_view(int64_t h) {
    wait(h);
    std::lock_guard<std::mutex> g(mu_);
    Spill& s = spills_.at(h);
    return at::from_blob(s.host, s.shape, at::TensorOptions().dtype(s.dtype).device(at::kCPU));
  }

  std::vector<int64_t> stats() {
    std::lock_guard<std::mutex> g(mu_);
    return {(int64_t)pool_.reserved(), (int64_t)pool_.used(), (int64_t)bytes_d2h_,
            (int64_t)bytes_h2d_, (int64_t)spills_.size()};
  }

 private:
  int device_;
  hipStream_t side_ = nullptr;
  PinnedPool pool_;
  std::map<int64_t, Spill> spills_;
  int64_t next_ = 1;
  size_t bytes_d2h_ = 0, bytes_h2d_ = 0;
  std::mutex mu_;
};

}  // namespace

TORCH_LIBRARY_FRAGMENT(tam, m) {
  m.class_<CkptEngine>("CkptEngine")
      .def(torch::init<int64_t, int64_t>())
      .def("spill", &CkptEngine::spill)
      .def("restore", &CkptEngine::restore)
      .def("ready", &CkptEngine::ready)
      .def("wait", &CkptEngine::wait)
      .def("release", &CkptEngine::release)
      .def("host_view", &CkptEngine::host_view)
      .def("copy_ms", &CkptEngine::copy_ms)
      .def("stream_handle", &CkptEngine::stream_handle)
      .def("stats", &CkptEngine::stats);
}
