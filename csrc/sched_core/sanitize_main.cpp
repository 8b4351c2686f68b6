// tiresias_amd — host-sanitizer driver for the native event core (SURVEY §5.2:
// "build the C++ control plane with -fsanitize=address,undefined").
//
// Built by tools/sanitize.sh / tests/test_sanitize.py with
//   g++ -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer
// and run on seeded synthetic traces for every policy the core supports.
// Besides the sanitizers' own checks it asserts the engine invariants the
// Python property tests pin: every job finishes, no job starts before it is
// submitted, JCT >= duration, no job ends before start + duration, and the
// GPU ledger returns to zero.
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

#include "engine.h"

namespace {

struct Lcg {   // deterministic, no <random> distribution differences across libstdc++
  unsigned long long s;
  double u() { s = s * 6364136223846793005ULL + 1442695040888963407ULL; return (double)(s >> 11) / 9007199254740992.0; }
};

int check(const char* pol, int n, int gpus, unsigned long long seed) {
  Lcg r{seed};
  std::vector<double> sub(n), dur(n);
  std::vector<int> g(n);
  double t = 0;
  for (int i = 0; i < n; ++i) {
    t += -std::log(1.0 - r.u()) * 40.0;
    sub[i] = t;
    dur[i] = 5.0 + std::exp(r.u() * 8.0);
    const double x = r.u();
    g[i] = x < 0.6 ? 1 : x < 0.75 ? 2 : x < 0.9 ? 4 : x < 0.97 ? 8 : 16;
    if (g[i] > gpus) g[i] = gpus;
  }
  std::vector<double> prior(dur.begin(), dur.end());
  tam_sched::Engine e(pol, gpus, {500.0, 5000.0}, std::string(pol).rfind("dlas", 0) == 0 ? 2.0 : 0.0,
                      300.0, prior);
  e.run(sub.data(), dur.data(), g.data(), n);
  int bad = 0;
  const auto& jobs = e.jobs();
  for (int i = 0; i < n; ++i) {
    const auto& j = jobs[i];
    const double tol = 1e-6 * (1.0 + j.end);
    if (j.state != tam_sched::DONE || j.start < j.submit - tol || j.end < j.start + j.dur - tol) {
      if (bad++ < 5)
        std::fprintf(stderr, "%s seed %llu job %d: state %d submit %.3f start %.3f end %.3f dur %.3f\n",
                     pol, seed, i, j.state, j.submit, j.start, j.end, j.dur);
    }
  }
  if (e.gpus_in_use() != 0) {
    std::fprintf(stderr, "%s: GPU ledger %ld != 0 after replay\n", pol, e.gpus_in_use());
    ++bad;
  }
  std::printf("%-18s n=%d gpus=%d seed=%llu events=%ld bad=%d\n", pol, n, gpus, seed, e.events(), bad);
  return bad;
}

}  // namespace

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 400;
  const char* pols[] = {"fifo", "fjf", "sjf", "shortest", "shortest-gpu", "dlas", "dlas-gpu",
                        "dlas-gpu-gittins", "gittins"};
  int bad = 0;
  for (const char* p : pols)
    for (unsigned long long seed = 1; seed <= 3; ++seed) bad += check(p, n, 16, seed);
  std::printf(bad ? "SANITIZE FAIL\n" : "SANITIZE OK\n");
  return bad ? 1 : 0;
}
