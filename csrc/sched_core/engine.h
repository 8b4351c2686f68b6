// tiresias_amd — native discrete-event core (engine only; no Python types).
// Included by the pybind11 module (sched_core.cpp) and by the host-sanitizer
// driver (sanitize_main.cpp: ASan + UBSan replay of every policy).
#pragma once
#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

namespace tam_sched {

constexpr double INF = std::numeric_limits<double>::infinity();
constexpr double EPS = 1e-9;

enum State { SUB = 0, PEND = 1, RUN = 2, DONE = 3 };

struct Job {
  double submit, dur;
  int gpu;
  long idx;
  double progress = 0, executed = 0, total_exec = 0, pending = 0, last_pending = 0;
  int q = 0;
  long seq = 0;
  double rank = 0;
  int state = SUB;
  double start = -1, end = -1, last_check = 0;
  int preempt = 0, resume = 0, promote = 0;
  double remaining() const { return std::max(0.0, dur - progress); }
  double attained(bool g) const { return g ? executed * gpu : executed; }
};

// Gittins index over a HISTORY sample (prior file), or -- online mode, no
// prior -- over the services of the jobs finished so far; rebuilt when the
// sample grew by 10 % (policy/las.py::GittinsTable applies the same rule).
struct Gittins {
  std::vector<double> samples, d, prefix;
  double delta = 1;
  size_t next_build = 0;
  void init(std::vector<double> data, double dl) {
    samples = std::move(data);
    delta = dl;
    build();
  }
  void build() {
    d = samples;
    std::sort(d.begin(), d.end());
    prefix.assign(d.size() + 1, 0.0);
    for (size_t i = 0; i < d.size(); ++i) prefix[i + 1] = prefix[i] + d[i];
    next_build = std::max(d.size() + 1, (size_t)((double)d.size() * 1.1));
  }
  void add(double s) {
    samples.push_back(s);
    if (samples.size() >= next_build) build();
  }
  double index(double a) const {
    const long n = (long)d.size();
    if (n == 0) return 0.0;
    const long i = std::upper_bound(d.begin(), d.end(), a) - d.begin();
    const long alive = n - i;
    if (alive <= 0) return 0.0;
    const long j = std::upper_bound(d.begin(), d.end(), a + delta) - d.begin();
    const long done = j - i;
    const double P = (double)done / (double)alive;
    const double E = ((prefix[j] - prefix[i]) - a * (double)done + delta * (double)(n - j)) / (double)alive;
    return E > 0 ? P / E : 0.0;
  }
};

enum Pol { FIFO, FJF, SJF, SRTF, SRSF, DLAS, DLASG, DLASGG, GITT };

inline Pol parse(const std::string& s) {
  if (s == "fifo") return FIFO;
  if (s == "fjf") return FJF;
  if (s == "sjf") return SJF;
  if (s == "shortest") return SRTF;
  if (s == "shortest-gpu") return SRSF;
  if (s == "dlas") return DLAS;
  if (s == "dlas-gpu") return DLASG;
  if (s == "dlas-gpu-gittins") return DLASGG;
  if (s == "gittins") return GITT;
  throw std::invalid_argument("sched_core: unsupported policy " + s);
}

class Engine {
 public:
  // online_prior: the prior starts empty and learns from finished jobs
  Engine(const std::string& policy, int total_gpus, std::vector<double> limits, double starve,
         double gittins_delta, std::vector<double> prior, bool online_prior = false)
      : pol_(parse(policy)), total_(total_gpus), limits_(std::move(limits)), starve_(starve),
        online_(online_prior) {
    std::sort(limits_.begin(), limits_.end());
    nq_ = (int)limits_.size() + 1;
    if (pol_ == DLASGG || pol_ == GITT) git_.init(std::move(prior), gittins_delta);
  }

  // Replays n jobs (arrays by job index); results are in jobs() afterwards.
  void run(const double* submit, const double* dur, const int* gpus, long n) {
    jobs_.clear();
    jobs_.reserve(n);
    for (long i = 0; i < n; ++i) {
      Job j;
      j.submit = submit[i]; j.dur = dur[i]; j.gpu = gpus[i]; j.idx = i;
      jobs_.push_back(j);
    }
    std::vector<long> order(n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](long a, long b) {
      return jobs_[a].submit < jobs_[b].submit;
    });
    cursor_ = 0;
    arrival_order_ = order;
    active_.clear();
    now_ = 0;
    used_ = 0;
    events_ = 0;
    long stall = 0;
    step(n ? std::min(next_arrival(), INF) : 0.0);
    while (true) {
      if (active_.empty() && cursor_ >= n) break;
      double t = next_time();
      if (t == INF) {
        for (long k : active_) if (jobs_[k].state == PEND) jobs_[k].state = -1;   // unplaceable
        break;
      }
      if (t <= now_ + 1e-9 * std::max(1.0, now_)) {
        t = now_;
        if (++stall > 10000) throw std::runtime_error("sched_core: no progress");
      } else {
        stall = 0;
      }
      step(t);
    }
  }

  const std::vector<Job>& jobs() const { return jobs_; }
  long events() const { return events_; }
  long gpus_in_use() const { return used_; }
  int total_gpus() const { return total_; }

 private:
  bool preemptive() const { return !(pol_ == FIFO || pol_ == FJF); }
  bool gputime() const { return pol_ != DLAS; }
  bool is_dlas() const { return pol_ == DLAS || pol_ == DLASG || pol_ == DLASGG; }

  double next_arrival() const {
    return cursor_ < (long)arrival_order_.size() ? jobs_[arrival_order_[cursor_]].submit : INF;
  }

  double next_time() {
    double t = next_arrival();
    for (long k : active_) {
      const Job& j = jobs_[k];
      if (j.state == RUN) t = std::min(t, now_ + j.remaining());
    }
    return std::min(t, policy_next());
  }

  double policy_next() {
    double t = INF;
    const bool g = gputime();
    for (long k : active_) {
      const Job& j = jobs_[k];
      if (is_dlas()) {
        if (j.state == RUN && j.q < nq_ - 1) {
          const double left = limits_[j.q] - j.attained(g);
          t = std::min(t, now_ + std::max(0.0, left) / (g ? j.gpu : 1));
        } else if (starve_ > 0 && j.state == PEND && j.q > 0 && j.executed > 0) {
          const double left = j.executed * starve_ - j.last_pending;
          if (left > 0) t = std::min(t, now_ + left);
        }
      }
      if ((pol_ == DLASGG || pol_ == GITT) && j.state == RUN) {
        const double dl = git_.delta;
        const double a = j.attained(true);
        const double nxt = (std::floor(a / dl + 1e-6) + 1) * dl;
        t = std::min(t, now_ + (nxt - a) / j.gpu);
      }
    }
    return t;
  }

  void advance(double t) {
    for (long k : active_) {
      Job& j = jobs_[k];
      const double dt = t - j.last_check;
      if (dt <= 0) continue;
      if (j.state == RUN) {
        j.total_exec += dt;
        j.executed += dt;
        j.progress = std::min(j.dur, j.progress + dt);
      } else if (j.state == PEND) {
        j.pending += dt;
        if (j.executed > 0) j.last_pending += dt;
      }
      j.last_check = t;
    }
    now_ = t;
  }

  void enter(Job& j, int q) { j.q = q; j.seq = ++seq_; }

  void step(double t) {
    advance(t);
    const double tol = 1e-9 * std::max(1.0, now_);
    for (size_t a = 0; a < active_.size();) {
      Job& j = jobs_[active_[a]];
      if (j.state == RUN && (j.remaining() <= EPS * std::max(1.0, j.dur) || j.remaining() <= tol)) {
        j.progress = j.dur;
        j.state = DONE;
        j.end = now_;
        used_ -= j.gpu;
        if (online_ && (pol_ == DLASGG || pol_ == GITT)) git_.add(j.total_exec * j.gpu);
        active_.erase(active_.begin() + a);
      } else {
        ++a;
      }
    }
    // arrivals within the clock tolerance of now (the loop snaps such events to now)
    while (cursor_ < (long)arrival_order_.size() && jobs_[arrival_order_[cursor_]].submit <= now_ + std::max(EPS, tol)) {
      Job& j = jobs_[arrival_order_[cursor_++]];
      j.state = PEND;
      j.last_check = now_;
      enter(j, 0);
      active_.push_back(j.idx);
    }
    update();
    schedule();
    if (is_dlas()) {
      std::vector<long> pend;
      for (long k : active_) if (jobs_[k].state == PEND) pend.push_back(k);
      std::sort(pend.begin(), pend.end(), [&](long a, long b) {
        const Job& x = jobs_[a]; const Job& y = jobs_[b];
        return x.q != y.q ? x.q < y.q : x.seq < y.seq;
      });
      for (long k : pend) jobs_[k].seq = ++seq_;
    }
    ++events_;
  }

  void update() {
    const bool g = gputime();
    // the same relative tolerance as the event clock: a threshold whose
    // remaining time rounds to "now" fires now instead of stalling the loop
    const double tol = 1e-9 * std::max(1.0, now_);
    for (long k : active_) {
      Job& j = jobs_[k];
      if (is_dlas()) {
        const double a = j.attained(g);
        if (j.state == RUN) {
          while (j.q < nq_ - 1 && a >= limits_[j.q] - tol * (g ? j.gpu : 1)) enter(j, j.q + 1);
        } else if (starve_ > 0 && j.state == PEND && j.q > 0 && j.executed > 0 &&
                   j.last_pending >= j.executed * starve_ - tol) {
          j.executed = 0; j.last_pending = 0; j.promote++;
          enter(j, 0);
        }
      }
      if (pol_ == DLASGG) j.rank = git_.index(j.attained(g));
      if (pol_ == GITT) j.rank = git_.index(j.attained(true));
    }
  }

  bool before(const Job& x, const Job& y) const {
    auto sub = [](const Job& a, const Job& b) { return a.submit != b.submit ? a.submit < b.submit : a.idx < b.idx; };
    const int rx = x.state == RUN ? 0 : 1, ry = y.state == RUN ? 0 : 1;
    switch (pol_) {
      case FIFO: case FJF: return sub(x, y);
      case SJF: return x.gpu != y.gpu ? x.gpu < y.gpu : sub(x, y);
      case SRTF: { const double a = x.remaining(), b = y.remaining(); return a != b ? a < b : sub(x, y); }
      case SRSF: { const double a = x.remaining() * x.gpu, b = y.remaining() * y.gpu; return a != b ? a < b : sub(x, y); }
      case DLAS: case DLASG:   // queue-entry order: demoted jobs queue behind pending ones
        if (x.q != y.q) return x.q < y.q;
        return x.seq < y.seq;
      case DLASGG:
        if (x.q != y.q) return x.q < y.q;
        if (x.rank != y.rank) return x.rank > y.rank;
        if (rx != ry) return rx < ry;
        return x.seq < y.seq;
      case GITT:
        if (x.rank != y.rank) return x.rank > y.rank;
        if (rx != ry) return rx < ry;
        return sub(x, y);
    }
    return false;
  }

  void start(Job& j) {
    if (j.start < 0) j.start = now_;
    j.state = RUN; j.resume++; j.last_check = now_;   // last_pending kept until promotion
    used_ += j.gpu;
  }
  void preempt(Job& j) {
    j.state = PEND; j.preempt++; j.last_check = now_;
    used_ -= j.gpu;
  }

  void schedule() {
    std::vector<long> ord;
    if (preemptive()) {
      ord = active_;
    } else {
      for (long k : active_) if (jobs_[k].state == PEND) ord.push_back(k);
    }
    std::stable_sort(ord.begin(), ord.end(), [&](long a, long b) { return before(jobs_[a], jobs_[b]); });
    if (preemptive()) {
      std::vector<char> chosen(jobs_.size(), 0);
      long used = 0;
      for (long k : ord) if (used + jobs_[k].gpu <= total_) { chosen[k] = 1; used += jobs_[k].gpu; }
      for (long k : active_) if (jobs_[k].state == RUN && !chosen[k]) preempt(jobs_[k]);
      for (long k : ord) if (chosen[k] && jobs_[k].state == PEND && jobs_[k].gpu <= total_ - used_) start(jobs_[k]);
      for (long k : ord)
        if (!chosen[k] && jobs_[k].state == PEND && jobs_[k].gpu <= total_ - used_) start(jobs_[k]);
    } else {
      for (long k : ord) {
        Job& j = jobs_[k];
        if (j.gpu <= total_ - used_) start(j);
        else if (pol_ == FIFO) break;
      }
    }
  }

  Pol pol_;
  int total_;
  bool online_ = false;
  std::vector<double> limits_;
  double starve_;
  int nq_;
  Gittins git_;
  std::vector<Job> jobs_;
  std::vector<long> arrival_order_, active_;
  long cursor_ = 0, seq_ = 0, events_ = 0;
  double now_ = 0;
  long used_ = 0;
};

}  // namespace tam_sched
