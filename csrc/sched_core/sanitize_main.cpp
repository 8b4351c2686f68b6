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

// The PRICED topology paths (round 5): yarn / tiresias placement on racks x
// nodes, checkpoint save / restore stalls (host, and HBM-resident with an
// xGMI copy on re-placement), the spread-gang network rate (measured
// slowdowns and the analytic all-reduce), and tiresias' wait-vs-spread rule.
// Same invariants as above, except that a priced job may end later than
// start + duration (its stalls and slower spread rate are the point).
int check_priced(const char* pol, const char* place, int ckpt, bool net, bool wait_rule, int n,
                 unsigned long long seed) {
  Lcg r{seed};
  const int switches = 2, nodes_per = 4, gpn = 8;
  const int gpus = switches * nodes_per * gpn;
  std::vector<double> sub(n), dur(n), ckb(n), sd(n), itc(n), nb(n);
  std::vector<int> g(n), gpw(n), tcpu(n), tmem(n);
  std::vector<unsigned char> sens(n);
  double t = 0;
  for (int i = 0; i < n; ++i) {
    t += -std::log(1.0 - r.u()) * 30.0;
    sub[i] = t;
    dur[i] = 5.0 + std::exp(r.u() * 8.0);
    const double x = r.u();
    g[i] = x < 0.55 ? 1 : x < 0.7 ? 2 : x < 0.85 ? 4 : x < 0.95 ? 8 : x < 0.99 ? 16 : 32;
    gpw[i] = 1;
    tcpu[i] = 4;
    tmem[i] = 16;
    sens[i] = r.u() < 0.3;                       // VGG-like placement-sensitive models
    ckb[i] = (0.2 + 3.0 * r.u()) * 1e9;          // state bytes per GPU
    sd[i] = r.u() < 0.5 ? 1.0 + r.u() : -1.0;    // measured 2-node slowdown, or analytic
    itc[i] = 0.01 + 0.2 * r.u();
    nb[i] = (20.0 + 500.0 * r.u()) * 1e6;
  }
  std::vector<double> prior(dur.begin(), dur.end());
  tam_sched::Engine e(pol, gpus, {500.0, 5000.0}, std::string(pol).rfind("dlas", 0) == 0 ? 2.0 : 0.0,
                      300.0, prior);
  e.set_topology(place, switches, nodes_per, gpn, 128, 512);
  tam_sched::Costs c;
  c.net = net;
  c.ckpt = ckpt;
  c.budget = 40e9;                               // small HBM budget: the over-budget host path runs too
  e.set_costs(c, ckb, sd, itc, nb);
  e.set_spread_wait(wait_rule);
  e.run_topo(sub.data(), dur.data(), g.data(), gpw.data(), tcpu.data(), tmem.data(), sens.data(), n);
  int bad = 0;
  const auto& jobs = e.jobs();
  for (int i = 0; i < n; ++i) {
    const auto& j = jobs[i];
    const double tol = 1e-6 * (1.0 + j.end);
    if (j.state != tam_sched::DONE || j.start < j.submit - tol || j.end < j.start + j.dur - tol ||
        !(j.overhead >= 0.0) || !std::isfinite(j.end)) {
      if (bad++ < 5)
        std::fprintf(stderr, "%s/%s ckpt %d net %d seed %llu job %d: state %d submit %.3f start %.3f end %.3f "
                     "dur %.3f overhead %.3f\n", pol, place, ckpt, (int)net, seed, i, j.state, j.submit,
                     j.start, j.end, j.dur, j.overhead);
    }
  }
  if (e.gpus_in_use() != 0) {
    std::fprintf(stderr, "%s/%s: GPU ledger %ld != 0 after replay\n", pol, place, e.gpus_in_use());
    ++bad;
  }
  std::printf("%-18s %-8s ckpt=%d net=%d wait=%d n=%d seed=%llu events=%ld spread=%ld wait=%ld bad=%d\n", pol,
              place, ckpt, (int)net, (int)wait_rule, n, seed, e.events(), e.spread_decisions(true),
              e.spread_decisions(false), bad);
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
  const char* priced_pols[] = {"fifo", "dlas-gpu", "gittins", "shortest"};
  for (const char* p : priced_pols)
    for (const char* place : {"yarn", "tiresias"})
      for (int ckpt = 0; ckpt <= 2; ++ckpt)
        for (int net = 0; net <= 1; ++net) {
          if (!net && !ckpt) continue;        // unpriced topology runs: covered by the spread row below
          bad += check_priced(p, place, ckpt, net, std::string(place) == "tiresias", n / 2, 7 + ckpt);
        }
  for (const char* p : priced_pols) bad += check_priced(p, "tiresias", 2, true, false, n / 2, 11);
  std::printf(bad ? "SANITIZE FAIL\n" : "SANITIZE OK\n");
  return bad ? 1 : 0;
}
