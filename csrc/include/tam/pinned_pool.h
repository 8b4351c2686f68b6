// tiresias_amd — first-fit host memory pool for checkpoint spills.
//
// Host-only code (no HIP in this header): the checkpoint engine instantiates
// it over pinned chunks (hipHostMalloc / hipHostFree), the sanitizer driver
// (csrc/sanitize/pool_sanitize_main.cpp) over malloc / free so ASan, UBSan and
// TSan exercise exactly the allocator logic the engine runs. Chunks are large
// (>= the configured chunk size), carved first-fit with coalescing on free,
// so a spill never calls the (synchronising, expensive) pinned allocator on
// the hot path once the pool is warm. Thread-safe: one mutex per pool.
#pragma once
#include <cstddef>
#include <mutex>
#include <stdexcept>
#include <vector>

namespace tam {

// AllocFn: void* (*)(size_t), FreeFn: void (*)(void*)
template <class AllocFn, class FreeFn>
class PinnedPool {
 public:
  PinnedPool(size_t chunk, AllocFn a, FreeFn f) : chunk_(chunk), alloc_(a), free_(f) {}
  PinnedPool(const PinnedPool&) = delete;
  PinnedPool& operator=(const PinnedPool&) = delete;
  ~PinnedPool() {
    for (auto& c : chunks_) free_(c.base);
  }

  static size_t round(size_t n) { return (n + 255) & ~size_t(255); }

  // returns a host pointer; grows by whole chunks (>= request)
  char* alloc(size_t n) {
    n = round(n == 0 ? 1 : n);
    std::lock_guard<std::mutex> g(mu_);
    for (auto& c : chunks_) {
      for (size_t i = 0; i < c.free.size(); ++i) {
        if (c.free[i].size >= n) {
          char* p = c.base + c.free[i].off;
          c.free[i].off += n;
          c.free[i].size -= n;
          if (c.free[i].size == 0) c.free.erase(c.free.begin() + (long)i);
          used_ += n;
          return p;
        }
      }
    }
    const size_t sz = n > chunk_ ? n : chunk_;
    Chunk c;
    c.base = static_cast<char*>(alloc_(sz));
    if (!c.base) throw std::bad_alloc();
    c.size = sz;
    if (sz > n) c.free.push_back({n, sz - n});
    chunks_.push_back(std::move(c));
    reserved_ += sz;
    used_ += n;
    return chunks_.back().base;
  }

  void free(char* p, size_t n) {
    n = round(n == 0 ? 1 : n);
    std::lock_guard<std::mutex> g(mu_);
    for (auto& c : chunks_) {
      if (p >= c.base && p < c.base + c.size) {
        if ((size_t)(p - c.base) + n > c.size) throw std::invalid_argument("PinnedPool: bad free size");
        Block b{(size_t)(p - c.base), n};
        auto it = c.free.begin();
        while (it != c.free.end() && it->off < b.off) ++it;
        if (it != c.free.end() && b.off + b.size > it->off) throw std::invalid_argument("PinnedPool: double free");
        if (it != c.free.begin() && (it - 1)->off + (it - 1)->size > b.off)
          throw std::invalid_argument("PinnedPool: double free");
        it = c.free.insert(it, b);
        if (it + 1 != c.free.end() && it->off + it->size == (it + 1)->off) {   // coalesce with next
          it->size += (it + 1)->size;
          c.free.erase(it + 1);
        }
        if (it != c.free.begin() && (it - 1)->off + (it - 1)->size == it->off) {   // with prev
          (it - 1)->size += it->size;
          c.free.erase(it);
        }
        used_ -= n;
        return;
      }
    }
    throw std::invalid_argument("PinnedPool: pointer not owned by pool");
  }

  size_t reserved() const { std::lock_guard<std::mutex> g(mu_); return reserved_; }
  size_t used() const { std::lock_guard<std::mutex> g(mu_); return used_; }
  // invariant: free blocks sorted, disjoint, inside their chunk; used + free == reserved
  bool check() const {
    std::lock_guard<std::mutex> g(mu_);
    size_t fr = 0;
    for (const auto& c : chunks_) {
      size_t end = 0;
      for (const auto& b : c.free) {
        if (b.off < end || b.off + b.size > c.size || b.size == 0) return false;
        end = b.off + b.size;
        fr += b.size;
      }
    }
    return fr + used_ == reserved_;
  }

 private:
  struct Block { size_t off, size; };
  struct Chunk { char* base = nullptr; size_t size = 0; std::vector<Block> free; };
  size_t chunk_;
  AllocFn alloc_;
  FreeFn free_;
  std::vector<Chunk> chunks_;
  size_t reserved_ = 0, used_ = 0;
  mutable std::mutex mu_;
};

}  // namespace tam
