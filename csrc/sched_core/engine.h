// tiresias_amd — native discrete-event core (engine only; no Python types).
// Included by the pybind11 module (sched_core.cpp) and by the host-sanitizer
// driver (sanitize_main.cpp: ASan + UBSan replay of every policy).
#pragma once
#include <algorithm>
#include <array>
#include <cmath>
#include <limits>
#include <map>
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
  // topology placement (yarn / tiresias): tasks of tgpu GPUs + tcpu / tmem,
  // placement-sensitivity (tiresias), and the committed plan:
  // per task [node, dev_0 .. dev_{tgpu-1}]
  int ntask = 1, tgpu = 1, tcpu = 0, tmem = 0;
  bool sens = false;
  std::vector<int> plan;
  std::vector<int> held;               // lazy preemption: plan of a tentatively released victim
  double progress = 0, executed = 0, total_exec = 0, pending = 0, last_pending = 0;
  int q = 0;
  long seq = 0;
  double rank = 0;
  int state = SUB;
  double start = -1, end = -1, last_check = 0;
  int preempt = 0, resume = 0, promote = 0;
  // priced replays (Engine::set_costs): progress rate of the current
  // placement (spread gangs < 1), the restore / save stall still ahead of
  // the next resume, and what checkpointing cost so far -- core/job.py
  double rate = 1.0, restore_left = 0.0, pending_ckpt = 0.0, overhead = 0.0, ckpt_bytes = 0.0;
  int where = 0;                       // suspended state: 0 none, 1 resident in HBM, 2 on the host
  std::vector<std::pair<int, int>> where_devs;   // (node, device) holding it when resident
  double remaining() const { return std::max(0.0, dur - progress); }
  double time_to_finish() const { return rate <= 0 ? INF : restore_left + remaining() / rate; }
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

// E[remaining service | attained a] over a service sample (GPU-seconds):
// engine/spread.py::ServiceEstimate (same rebuild rule when learned online)
struct ServiceEst {
  std::vector<double> raw, d, pre{0.0};
  size_t next = 0;
  void init(const std::vector<double>& s) {
    raw = s;
    if (!raw.empty()) build();
  }
  void build() {
    d = raw;
    std::sort(d.begin(), d.end());
    pre.assign(1, 0.0);
    for (double x : d) pre.push_back(pre.back() + x);
    next = std::max(d.size() + 1, (size_t)((double)d.size() * 1.1));
  }
  void add(double s) {
    raw.push_back(s);
    if (raw.size() >= next) build();
  }
  bool empty() const { return d.empty(); }
  double remaining(double a) const {
    const size_t n = d.size();
    const size_t i = std::upper_bound(d.begin(), d.end(), a) - d.begin();
    const size_t alive = n - i;
    if (alive == 0) return std::max(a, pre[n] / (double)n);
    return (pre[n] - pre[i]) / (double)alive - a;
  }
};

enum Pol { FIFO, FJF, SJF, SRTF, SRSF, DLAS, DLASG, DLASGG, GITT };
// P_COUNT: flat GPU pool; P_FILL: "count" on the topology (placement/
// schemes.py::CountPlacement: tasks filled node by node in id order) -- used
// when costs need the nodes / devices a job landed on
enum Place { P_COUNT, P_YARN, P_TIRESIAS, P_FILL };

inline Place parse_place(const std::string& s) {
  if (s.empty()) return P_COUNT;
  if (s == "count") return P_FILL;
  if (s == "yarn") return P_YARN;
  if (s == "tiresias") return P_TIRESIAS;
  throw std::invalid_argument("sched_core: unsupported placement " + s);
}

// The Python engine's cost terms (engine/sim.py::Simulator._rate and
// engine/ckpt_model.py::CkptCostModel), evaluated from per-job parameters the
// front-end derives once (engine/native.py):
//  * network: a gang spread over k > 1 nodes progresses at
//    1 / (1 + (sd - 1) * 2(k-1)/k) from its MEASURED 2-node slowdown sd
//    (cluster/network.py::measured_spread_rate), else c / (c + allreduce(k))
//    with per-iteration time c and the analytic ring all-reduce over the
//    link bandwidth / latency (network_rate);
//  * checkpoints: 0 none; 1 host (every preemption spills, every resume
//    restores: bytes / bandwidth); 2 hbm / measured / pressure (suspended
//    state stays resident within a per-GPU budget: resume on the same GPUs
//    free, elsewhere an xGMI copy; over budget the host path).
struct Costs {
  bool net = false;
  double bw_mbps = 1250.0, latency = 0.015;
  int ckpt = 0;
  double host_gbps = 50.0, h2d_gbps = 50.0, xgmi_gbps = 64.0, budget = 200e9;
};

// Racks x nodes x devices with per-node CPU / memory, the Python Cluster's
// exclusive (no packing) state: cluster/topology.py. Placement plans are
// built on a scratch copy and committed atomically, as there.
struct Topo {
  int gpn = 0;
  std::vector<int> rack;                        // node -> rack
  std::vector<std::vector<int>> rack_nodes;     // rack -> its nodes, in node order
  std::vector<int> cpu_cap, mem_cap, cpu_used, mem_used;
  std::vector<std::vector<char>> busy;          // node -> device busy
  void init(int switches, int nodes_per, int gpus, int cpus, int mem) {
    gpn = gpus;
    const int n = switches * nodes_per;
    rack.assign(n, 0);
    rack_nodes.assign(switches, {});
    for (int i = 0; i < n; ++i) { rack[i] = i / nodes_per; rack_nodes[i / nodes_per].push_back(i); }
    cpu_cap.assign(n, cpus); mem_cap.assign(n, mem);
    cpu_used.assign(n, 0); mem_used.assign(n, 0);
    busy.assign(n, std::vector<char>(gpus, 0));
  }
  int nodes() const { return (int)busy.size(); }
  int nfree(int n) const {
    int c = 0;
    for (char b : busy[n]) c += !b;
    return c;
  }
};

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
    svc_online_ = prior.empty();
    svc_init_ = prior;
    if (pol_ == DLASGG || pol_ == GITT) git_.init(std::move(prior), gittins_delta);
  }

  // tiresias placement, insensitive gangs: false = fragments first (spread
  // whenever no consolidated block is free), true = wait-vs-spread
  // (engine/spread.py; needs set_costs' per-job spread parameters)
  void set_spread_wait(bool on) { spread_wait_ = on; }
  // spread_rule "node": a gang that fits one node is never fragmented across
  // nodes (it waits for a free node; the wait-vs-spread rule decides only
  // for gangs wider than a node)
  void set_spread_node(bool on) { spread_node_ = on; }
  // spread_rule "price": the wait-vs-spread penalty also charges the queued
  // gangs whose consolidated block the spread's fragments delay
  // (engine/spread.py::SpreadAdvisor.fragment_cost)
  void set_spread_price(bool on) { spread_price_ = on; }
  // preemptive policies on topology placements: lazy (default) or eager
  void set_lazy_preempt(bool on) { lazy_ = on; }
  long spread_decisions(bool spread) const { return spread ? n_spread_ : n_wait_; }

  // Topology placement (yarn / tiresias) on switches x nodes x gpus with
  // per-node CPU / memory; per-job task shape and sensitivity are passed to
  // run_topo. "count" keeps the flat GPU pool.
  void set_topology(const std::string& placement, int switches, int nodes_per, int gpus, int cpus, int mem) {
    place_ = parse_place(placement);
    topo_.init(switches, nodes_per, gpus, cpus, mem);
    total_ = switches * nodes_per * gpus;
  }

  // Cost terms (see Costs) and their per-job parameters: state bytes per GPU
  // (ckpt_b), measured 2-node slowdown (net_sd, < 0: none -> analytic with
  // per-iteration seconds net_c and all-reduce bytes net_bytes). Arrays of
  // the next run's length; costs need a topology placement.
  void set_costs(const Costs& c, std::vector<double> ckpt_b, std::vector<double> net_sd,
                 std::vector<double> net_c, std::vector<double> net_bytes) {
    costs_ = c;
    ckpt_b_ = std::move(ckpt_b); net_sd_ = std::move(net_sd);
    net_c_ = std::move(net_c); net_bytes_ = std::move(net_bytes);
  }
  bool priced() const { return costs_.net || costs_.ckpt != 0; }

  void run_topo(const double* submit, const double* dur, const int* gpus, const int* gpw, const int* tcpu,
                const int* tmem, const unsigned char* sens, long n) {
    shape_.assign(n, {});
    for (long i = 0; i < n; ++i) {
      const int w = std::max(1, gpw[i]);
      shape_[i] = {std::max(1, gpus[i] / w), w, tcpu[i], tmem[i], (int)sens[i]};
    }
    run(submit, dur, gpus, n);
  }

  // Replays n jobs (arrays by job index); results are in jobs() afterwards.
  void run(const double* submit, const double* dur, const int* gpus, long n) {
    jobs_.clear();
    jobs_.reserve(n);
    for (long i = 0; i < n; ++i) {
      Job j;
      j.submit = submit[i]; j.dur = dur[i]; j.gpu = gpus[i]; j.idx = i;
      if (place_ != P_COUNT) {
        if ((long)shape_.size() != n) throw std::invalid_argument("sched_core: run_topo needs per-job shapes");
        j.ntask = shape_[i][0]; j.tgpu = shape_[i][1]; j.tcpu = shape_[i][2]; j.tmem = shape_[i][3];
        j.sens = shape_[i][4] != 0;
      }
      jobs_.push_back(j);
    }
    if (priced()) {
      if (place_ == P_COUNT) throw std::invalid_argument("sched_core: costs need a topology placement");
      if ((long)ckpt_b_.size() != n || (long)net_sd_.size() != n || (long)net_c_.size() != n ||
          (long)net_bytes_.size() != n)
        throw std::invalid_argument("sched_core: set_costs arrays must match the run's job count");
    }
    resident_.clear();
    svc_ = ServiceEst();
    svc_.init(svc_init_);
    n_spread_ = n_wait_ = 0;
    if (spread_wait_ && place_ == P_TIRESIAS && (long)net_sd_.size() != n)
      throw std::invalid_argument("sched_core: the wait spread rule needs set_costs' per-job arrays");
    if (place_ != P_COUNT) {
      for (int k = 0; k < topo_.nodes(); ++k) {
        std::fill(topo_.busy[k].begin(), topo_.busy[k].end(), 0);
        topo_.cpu_used[k] = 0; topo_.mem_used[k] = 0;
      }
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
        if (++stall > 10000) throw std::runtime_error("sched_core: no progress (" + stall_info() + ")");
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
      if (j.state == RUN) t = std::min(t, now_ + j.time_to_finish());
    }
    return std::min(t, policy_next());
  }

  // wall seconds to the job's next Gittins quantum boundary; one closer than
  // the clock tolerance counts as reached (policy/las.py::_quantum_wait)
  double quantum_wait(const Job& j) const {
    const double dl = git_.delta;
    const double a = j.attained(true);
    double w = ((std::floor(a / dl + 1e-6) + 1) * dl - a) / j.gpu;
    if (w <= 1e-9 * std::max(1.0, now_)) w += dl / j.gpu;
    return w;
  }

  // what keeps requesting events at now (the stall diagnostic)
  std::string stall_info() {
    std::string out = "t=" + std::to_string(now_);
    for (long k : active_) {
      const Job& j = jobs_[k];
      if (j.state == RUN && now_ + j.time_to_finish() <= now_ + 1e-9 * std::max(1.0, now_))
        out += " finish:job" + std::to_string(j.idx) + " ttf=" + std::to_string(j.time_to_finish()) +
               " rem=" + std::to_string(j.remaining()) + " rate=" + std::to_string(j.rate);
    }
    const double p = policy_next();
    out += " policy_next-now=" + std::to_string(p - now_);
    return out;
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
      if ((pol_ == DLASGG || pol_ == GITT) && j.state == RUN) t = std::min(t, now_ + quantum_wait(j));
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
        double work = dt;
        if (j.restore_left > 0) {                 // stalled on a restore / the last save
          const double r = std::min(j.restore_left, dt);
          j.restore_left -= r;
          work -= r;
        }
        j.progress = std::min(j.dur, j.progress + work * j.rate);
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
      if (j.state == RUN && (j.remaining() <= EPS * std::max(1.0, j.dur) || j.time_to_finish() <= tol)) {
        j.progress = j.dur;
        j.state = DONE;
        j.end = now_;
        used_ -= j.gpu;
        release(j);
        ckpt_finish(j);
        if (svc_online_) svc_.add(j.total_exec * j.gpu);
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
    if (costs_.net) refresh_rates();
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
    if (priced()) {
      // stall before progress resumes: this restore + the last preemption's save
      const double restore = ckpt_resume(j);
      j.restore_left = restore + j.pending_ckpt;
      j.pending_ckpt = 0;
      j.overhead += restore;
      j.rate = 1.0;                                  // refresh_rates after the round
    }
  }
  void preempt(Job& j) {
    if (priced()) {
      const double save = ckpt_preempt(j);          // on the allocation it ran on
      j.restore_left = 0;
      j.pending_ckpt += save;
      j.overhead += save;
    }
    j.state = PEND; j.preempt++; j.last_check = now_;
    used_ -= j.gpu;
    release(j);
  }

  // ------------------------------------------------------------ cost terms
  std::vector<std::pair<int, int>> devs_of(const Job& j) const {
    std::vector<std::pair<int, int>> v;
    size_t p = 0;
    for (int t = 0; t < j.ntask && p < j.plan.size(); ++t) {
      const int nd = j.plan[p++];
      for (int g = 0; g < j.tgpu; ++g) v.emplace_back(nd, j.plan[p++]);
    }
    std::sort(v.begin(), v.end());
    return v;
  }
  int nodes_of(const Job& j) const {
    std::vector<int> nd;
    size_t p = 0;
    for (int t = 0; t < j.ntask && p < j.plan.size(); ++t) {
      nd.push_back(j.plan[p]);
      p += 1 + j.tgpu;
    }
    std::sort(nd.begin(), nd.end());
    return (int)(std::unique(nd.begin(), nd.end()) - nd.begin());
  }
  double spread_rate(const Job& j, int k) const {
    if (k <= 1) return 1.0;
    const double sd = net_sd_[j.idx];
    if (sd >= 0) return 1.0 / (1.0 + std::max(0.0, sd - 1.0) * 2.0 * (k - 1) / k);
    const double c = net_c_[j.idx];
    const double comm = 2.0 * (k - 1) / k * (net_bytes_[j.idx] / 1048576.0) / costs_.bw_mbps +
                        2.0 * (k - 1) * costs_.latency;
    return c > 0 ? c / (c + comm) : 1.0;
  }
  void refresh_rates() {
    for (long k : active_) {
      Job& j = jobs_[k];
      if (j.state == RUN) j.rate = spread_rate(j, nodes_of(j));
    }
  }
  // engine/ckpt_model.py::CkptCostModel.on_preempt -> save seconds
  double ckpt_preempt(Job& j) {
    j.where = 0;
    if (costs_.ckpt == 0) return 0.0;
    const double b = ckpt_b_[j.idx];
    if (costs_.ckpt == 2 && !j.plan.empty()) {
      const auto devs = devs_of(j);
      bool fits = true;
      for (const auto& d : devs) {
        auto it = resident_.find(d);
        if ((it == resident_.end() ? 0.0 : it->second) + b > costs_.budget) { fits = false; break; }
      }
      if (fits) {
        for (const auto& d : devs) resident_[d] += b;
        j.where = 1;
        j.where_devs = devs;
        return 0.0;
      }
    }
    j.where = 2;
    j.where_devs.clear();
    j.ckpt_bytes += b * j.gpu;
    return b / (costs_.host_gbps * 1e9);
  }
  void unreside(Job& j, double b) {
    for (const auto& d : j.where_devs) {
      double& r = resident_[d];
      r = std::max(0.0, r - b);
    }
    j.where_devs.clear();
  }
  // on_resume -> restore seconds (the job's new plan is committed)
  double ckpt_resume(Job& j) {
    const int w = j.where;
    j.where = 0;
    if (w == 0 || costs_.ckpt == 0) return 0.0;
    const double b = ckpt_b_[j.idx];
    if (w == 1) {
      const bool same = j.where_devs == devs_of(j);
      unreside(j, b);
      if (same) return 0.0;
      j.ckpt_bytes += b * j.gpu;
      return b / (costs_.xgmi_gbps * 1e9);
    }
    j.ckpt_bytes += b * j.gpu;
    return b / (costs_.h2d_gbps * 1e9);
  }
  void ckpt_finish(Job& j) {
    if (j.where == 1) unreside(j, ckpt_b_.empty() ? 0.0 : ckpt_b_[j.idx]);
    j.where = 0;
  }

  // ------------------------------------------------------------ placement
  // engine/sim.py::Simulator._try_place -> placement/schemes.py
  bool try_place(Job& j) {
    if (j.gpu > total_) return false;
    if (place_ == P_COUNT) {
      if (j.gpu > total_ - used_) return false;
      start(j);
      return true;
    }
    std::vector<int> plan;
    bool ok;
    if (place_ == P_FILL) {
      std::vector<int> all(topo_.nodes());
      std::iota(all.begin(), all.end(), 0);
      ok = fill(j, all, plan);
    } else {
      ok = place_ == P_YARN ? plan_yarn(j, plan) : plan_tiresias(j, plan);
    }
    if (!ok) return false;
    commit(j, plan);
    start(j);
    return true;
  }

  void commit(Job& j, const std::vector<int>& plan) {
    j.plan = plan;
    size_t p = 0;
    for (int t = 0; t < j.ntask; ++t) {
      const int nd = plan[p++];
      topo_.cpu_used[nd] += j.tcpu;
      topo_.mem_used[nd] += j.tmem;
      for (int g = 0; g < j.tgpu; ++g) topo_.busy[nd][plan[p++]] = 1;
    }
  }

  void release(Job& j) {
    if (place_ == P_COUNT || j.plan.empty()) return;
    size_t p = 0;
    for (int t = 0; t < j.ntask; ++t) {
      const int nd = j.plan[p++];
      topo_.cpu_used[nd] -= j.tcpu;
      topo_.mem_used[nd] -= j.tmem;
      for (int g = 0; g < j.tgpu; ++g) topo_.busy[nd][j.plan[p++]] = 0;
    }
    j.plan.clear();
  }

  // placement/schemes.py::_fill on a scratch view: each task on the first
  // node of ``order`` with the CPU / memory and tgpu free devices (lowest ids)
  bool fill(const Job& j, const std::vector<int>& order, std::vector<int>& plan) const {
    plan.clear();
    std::vector<int> cpu = topo_.cpu_used, mem = topo_.mem_used;
    std::vector<std::vector<char>> busy;   // copied lazily per touched node
    std::vector<int> copied(topo_.nodes(), -1);
    auto dev_busy = [&](int nd, int d) {
      return copied[nd] >= 0 ? busy[copied[nd]][d] : topo_.busy[nd][d];
    };
    for (int t = 0; t < j.ntask; ++t) {
      bool placed = false;
      for (int nd : order) {
        if (topo_.cpu_cap[nd] - cpu[nd] < j.tcpu || topo_.mem_cap[nd] - mem[nd] < j.tmem) continue;
        int have = 0;
        for (int d = 0; d < topo_.gpn; ++d) have += !dev_busy(nd, d);
        if (have < j.tgpu) continue;
        if (copied[nd] < 0) { copied[nd] = (int)busy.size(); busy.push_back(topo_.busy[nd]); }
        auto& b = busy[copied[nd]];
        plan.push_back(nd);
        int got = 0;
        for (int d = 0; d < topo_.gpn && got < j.tgpu; ++d)
          if (!b[d]) { b[d] = 1; plan.push_back(d); ++got; }
        cpu[nd] += j.tcpu; mem[nd] += j.tmem;
        placed = true;
        break;
      }
      if (!placed) return false;
    }
    return true;
  }

  bool single_node(const Job& j, const std::vector<int>& order, std::vector<int>& plan) const {
    for (int nd : order) {
      if (fill(j, {nd}, plan)) return true;
    }
    return false;
  }

  // placement/schemes.py::YarnPlacement
  bool plan_yarn(const Job& j, std::vector<int>& plan) const {
    const int N = topo_.nodes();
    if (j.gpu <= topo_.gpn) {
      std::vector<int> order(N);
      std::iota(order.begin(), order.end(), 0);
      return single_node(j, order, plan);
    }
    auto by_free = [&](std::vector<int> v) {
      std::stable_sort(v.begin(), v.end(), [&](int a, int b) { return topo_.nfree(a) > topo_.nfree(b); });
      return v;
    };
    for (const auto& rn : topo_.rack_nodes) {
      std::vector<int> nodes = by_free(rn);
      int tot = 0;
      for (int nd : nodes) tot += topo_.nfree(nd);
      if (tot >= j.gpu && fill(j, nodes, plan)) return true;
    }
    std::vector<int> all(N);
    std::iota(all.begin(), all.end(), 0);
    return fill(j, by_free(all), plan);
  }

  // placement/schemes.py::TiresiasPlacement._exclusive (skew-aware)
  bool plan_tiresias(const Job& j, std::vector<int>& plan) const {
    const int N = topo_.nodes(), gpn = topo_.gpn;
    std::vector<int> all(N);
    std::iota(all.begin(), all.end(), 0);
    if (j.sens) {
      if (j.gpu <= gpn) {
        std::vector<int> order = all;
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
          const int fa = topo_.nfree(a), fb = topo_.nfree(b);
          return fa != fb ? fa < fb : a < b;
        });
        return single_node(j, order, plan);
      }
      std::vector<int> whole;
      for (int nd : all) if (topo_.nfree(nd) == gpn) whole.push_back(nd);
      if ((long)whole.size() * gpn < j.gpu) return false;
      std::vector<int> rk;                         // racks by first appearance in ``whole``
      std::vector<std::vector<int>> groups;
      for (int nd : whole) {
        const int r = topo_.rack[nd];
        auto it = std::find(rk.begin(), rk.end(), r);
        if (it == rk.end()) { rk.push_back(r); groups.push_back({nd}); }
        else groups[it - rk.begin()].push_back(nd);
      }
      std::vector<int> gi(groups.size());
      std::iota(gi.begin(), gi.end(), 0);
      std::stable_sort(gi.begin(), gi.end(), [&](int a, int b) { return groups[a].size() > groups[b].size(); });
      for (int g : gi)
        if ((long)groups[g].size() * gpn >= j.gpu) return fill(j, groups[g], plan);
      return fill(j, whole, plan);
    }
    std::vector<int> order = all;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
      const int fa = topo_.nfree(a), fb = topo_.nfree(b);
      if ((fa == 0) != (fb == 0)) return fa != 0;
      return fa != fb ? fa < fb : a < b;
    });
    if (!spread_wait_) return fill(j, order, plan);
    // wait-vs-spread (placement/schemes.py::TiresiasPlacement._exclusive)
    if (j.gpu <= gpn) {
      std::vector<int> best = all;
      std::stable_sort(best.begin(), best.end(), [&](int a, int b) {
        const int fa = topo_.nfree(a), fb = topo_.nfree(b);
        return fa != fb ? fa < fb : a < b;
      });
      if (single_node(j, best, plan)) return true;
      if (spread_node_) return false;
    } else if (spread_node_) {   // wider than a node: fullest-free nodes first
      std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        const int fa = topo_.nfree(a), fb = topo_.nfree(b);
        return fa != fb ? fa > fb : a < b;
      });
    }
    if (!fill(j, order, plan)) return false;
    std::vector<int> nd;
    for (size_t p = 0; p < plan.size(); p += 1 + j.tgpu) nd.push_back(plan[p]);
    std::sort(nd.begin(), nd.end());
    const int k = (int)(std::unique(nd.begin(), nd.end()) - nd.begin());
    const int min_nodes = std::max(1, (j.gpu + gpn - 1) / gpn);
    if (k <= min_nodes || should_spread(j, k, min_nodes)) return true;
    plan.clear();
    return false;
  }

  // engine/spread.py::SpreadAdvisor (the engine's remaining-wall / rate rules)
  bool remaining_wall(const Job& j, double& out) const {
    if (svc_.empty()) return false;
    const double rem = svc_.remaining(j.attained(true));
    const double r = (j.state == RUN && j.rate > 0) ? j.rate : 1.0;
    out = rem / std::max(1, j.gpu) / r + (j.state == RUN ? j.restore_left : 0.0);
    return true;
  }
  double wait_for_block(const Job& j, int min_nodes) const {
    const int N = topo_.nodes(), gpn = topo_.gpn;
    std::vector<std::vector<std::pair<double, int>>> per(N);
    for (long k : active_) {
      const Job& r = jobs_[k];
      if (r.state != RUN || r.plan.empty()) continue;
      double rem = 0;
      remaining_wall(r, rem);
      std::vector<int> cnt(N, 0);
      size_t p = 0;
      for (int t = 0; t < r.ntask; ++t) { cnt[r.plan[p]] += r.tgpu; p += 1 + r.tgpu; }
      for (int nd = 0; nd < N; ++nd) if (cnt[nd]) per[nd].emplace_back(rem, cnt[nd]);
    }
    const bool whole = j.gpu > gpn;
    std::vector<double> times;
    for (int nd = 0; nd < N; ++nd) {
      if (whole) {
        double m = 0.0;
        for (const auto& e : per[nd]) m = std::max(m, e.first);
        times.push_back(m);
        continue;
      }
      if (gpn < j.gpu) continue;
      int free = topo_.nfree(nd);
      double t = 0.0;
      std::sort(per[nd].begin(), per[nd].end());
      for (const auto& e : per[nd]) {
        if (free >= j.gpu) break;
        free += e.second;
        t = e.first;
      }
      if (free >= j.gpu) times.push_back(t);
    }
    if (whole) {
      std::sort(times.begin(), times.end());
      return (int)times.size() >= min_nodes ? times[min_nodes - 1] : INF;
    }
    double m = INF;
    for (double t : times) m = std::min(m, t);
    return m;
  }
  // engine/spread.py::SpreadAdvisor.fragment_cost (terms summed ascending)
  double fragment_cost(const Job& j, double hold_s) const {
    const int gpn = topo_.gpn;
    std::vector<double> terms;
    for (long k : active_) {
      const Job& q = jobs_[k];
      if (&q == &j || q.state != PEND || q.gpu < 2) continue;
      const double w = wait_for_block(q, std::max(1, (q.gpu + gpn - 1) / gpn));
      if (w < hold_s) terms.push_back((hold_s - w) * q.gpu / (double)std::max(1, j.gpu));
    }
    std::sort(terms.begin(), terms.end());
    double s = 0.0;
    for (double t : terms) s += t;
    return s;
  }
  bool should_spread(const Job& j, int k, int min_nodes) const {
    const double r_k = spread_rate(j, k), r_min = spread_rate(j, min_nodes);
    double rem = 0;
    bool ok;
    if (!remaining_wall(j, rem) || r_k <= 0) {
      ok = true;
    } else {
      double penalty = (1.0 / r_k - 1.0 / std::max(r_min, 1e-9)) * rem;
      if (spread_price_) penalty += fragment_cost(j, rem / r_k);
      ok = wait_for_block(j, min_nodes) > penalty;
    }
    ++(ok ? n_spread_ : n_wait_);
    return ok;
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
      if (lazy_ && (place_ == P_YARN || place_ == P_TIRESIAS)) {   // "count" stays eager (Python: the same)
        schedule_lazy(ord, chosen);
        return;
      }
      for (long k : active_) if (jobs_[k].state == RUN && !chosen[k]) preempt(jobs_[k]);
      for (long k : ord) if (chosen[k] && jobs_[k].state == PEND) try_place(jobs_[k]);
      // work-conserving back-fill (chosen jobs that failed placement are not retried)
      if (total_ - used_ > 0)
        for (long k : ord)
          if (!chosen[k] && jobs_[k].state == PEND && jobs_[k].gpu <= total_ - used_) try_place(jobs_[k]);
    } else {
      for (long k : ord) {
        if (!try_place(jobs_[k]) && pol_ == FIFO) break;
      }
    }
  }

  // engine/sim.py::Simulator._schedule_lazy (topology placements): victims
  // released tentatively, chosen jobs placed, then the back-fill in priority
  // order re-commits a victim whose devices are all still free in place and
  // preempts the others (which may then be placed elsewhere, as any pending job)
  bool plan_free(const Job& j, const std::vector<int>& plan) const {
    std::vector<int> cpu = topo_.cpu_used, mem = topo_.mem_used;
    size_t p = 0;
    for (int t = 0; t < j.ntask; ++t) {
      const int nd = plan[p++];
      cpu[nd] += j.tcpu; mem[nd] += j.tmem;
      if (cpu[nd] > topo_.cpu_cap[nd] || mem[nd] > topo_.mem_cap[nd]) return false;
      for (int g = 0; g < j.tgpu; ++g) if (topo_.busy[nd][plan[p++]]) return false;
    }
    return true;
  }
  void schedule_lazy(const std::vector<long>& ord, const std::vector<char>& chosen) {
    std::vector<long> victims;
    for (long k : ord) if (jobs_[k].state == RUN && !chosen[k]) victims.push_back(k);
    for (long k : victims) {
      Job& v = jobs_[k];
      v.held = v.plan;
      release(v);                                  // topology free, still RUN
      used_ -= v.gpu;
    }
    for (long k : ord) if (chosen[k] && jobs_[k].state == PEND) try_place(jobs_[k]);
    for (long k : ord) {
      Job& j = jobs_[k];
      if (!j.held.empty()) {
        std::vector<int> h;
        h.swap(j.held);
        if (plan_free(j, h)) {                     // nothing took its GPUs: it never stopped
          commit(j, h);
          used_ += j.gpu;
          continue;
        }
        j.plan = h;                                // preempt on the allocation it ran on
        if (priced()) {
          const double save = ckpt_preempt(j);
          j.restore_left = 0;
          j.pending_ckpt += save;
          j.overhead += save;
        }
        j.state = PEND; j.preempt++; j.last_check = now_;
        j.plan.clear();                            // (topology and ledger already released)
      }
      if (j.state == PEND && !chosen[k] && j.gpu > 0 && j.gpu <= total_ - used_) try_place(j);
    }
  }

  Pol pol_;
  bool lazy_ = true;
  Place place_ = P_COUNT;
  Costs costs_;
  bool spread_wait_ = false, spread_node_ = false, spread_price_ = false, svc_online_ = true;
  std::vector<double> svc_init_;
  ServiceEst svc_;
  mutable long n_spread_ = 0, n_wait_ = 0;
  std::vector<double> ckpt_b_, net_sd_, net_c_, net_bytes_;
  std::map<std::pair<int, int>, double> resident_;   // (node, device) -> suspended state bytes
  Topo topo_;
  std::vector<std::array<int, 5>> shape_;
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
