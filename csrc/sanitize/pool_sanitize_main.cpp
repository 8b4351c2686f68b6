// tiresias_amd — host-sanitizer driver for the checkpoint engine's pinned pool
// (SURVEY §5.2). Built by tools/sanitize.sh twice: -fsanitize=address,undefined
// and -fsanitize=thread. Several threads spill / release concurrently (the
// engine is called from the worker thread while a recovery or status thread
// may release), with randomized sizes; every owner writes and re-checks a
// byte pattern over its block (overlap = corruption), and the pool invariant
// (free blocks disjoint, used + free == reserved) is checked at the end.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "tam/pinned_pool.h"

namespace {
void* host_alloc(size_t n) { return std::malloc(n); }
void host_free(void* p) { std::free(p); }
using Pool = tam::PinnedPool<void* (*)(size_t), void (*)(void*)>;

std::atomic<int> errors{0};

void worker(Pool* pool, int tid, int iters) {
  unsigned long long s = 0x9e3779b97f4a7c15ULL * (unsigned)(tid + 1);
  auto rnd = [&]() { s = s * 6364136223846793005ULL + 1442695040888963407ULL; return (unsigned)(s >> 33); };
  struct Own { char* p; size_t n; unsigned char tag; };
  std::vector<Own> own;
  for (int i = 0; i < iters; ++i) {
    if (own.empty() || rnd() % 3 != 0) {
      const size_t n = 1 + rnd() % (1u << (8 + rnd() % 12));
      char* p = pool->alloc(n);
      const unsigned char tag = (unsigned char)(tid * 31 + i);
      std::memset(p, tag, n);
      own.push_back({p, n, tag});
    } else {
      const size_t k = rnd() % own.size();
      Own o = own[k];
      for (size_t b = 0; b < o.n; ++b)
        if ((unsigned char)o.p[b] != o.tag) { errors++; break; }
      pool->free(o.p, o.n);
      own.erase(own.begin() + (long)k);
    }
  }
  for (auto& o : own) {
    for (size_t b = 0; b < o.n; ++b)
      if ((unsigned char)o.p[b] != o.tag) { errors++; break; }
    pool->free(o.p, o.n);
  }
}
}  // namespace

int main(int argc, char** argv) {
  const int threads = argc > 1 ? std::atoi(argv[1]) : 4;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 3000;
  Pool pool(1 << 20, host_alloc, host_free);
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) ts.emplace_back(worker, &pool, t, iters);
  for (auto& t : ts) t.join();
  if (!pool.check() || pool.used() != 0 || errors.load() != 0) {
    std::printf("POOL FAIL used=%zu errors=%d\n", pool.used(), errors.load());
    return 1;
  }
  bool threw = false;
  try { pool.free(reinterpret_cast<char*>(&threw), 8); } catch (const std::invalid_argument&) { threw = true; }
  if (!threw) { std::printf("POOL FAIL: foreign pointer accepted\n"); return 1; }
  std::printf("POOL OK reserved=%zu threads=%d iters=%d\n", pool.reserved(), threads, iters);
  return 0;
}
