// tiresias_amd — native discrete-event core for full-trace replays.
//
// The Python engine (tiresias_amd/engine/sim.py) models everything (topology
// placements, packing, interference, network, checkpoints, live runtime);
// it is O(active jobs) Python per event. Replaying the month-long NSDI'19
// trace (~10^5 jobs) across a policy sweep needs a native loop. This core
// implements the same event semantics for the count / yarn / tiresias
// placements with the preemptive / non-preemptive policy family Tiresias is
// evaluated on — fifo, fjf, sjf, shortest, shortest-gpu, dlas, dlas-gpu,
// dlas-gpu-gittins, gittins — optionally PRICED like the Python engine
// (spread-gang network rate, checkpoint save / restore stalls: set_costs),
// and is cross-checked job-for-job against the Python engine in
// tests/test_sched_core.py.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "engine.h"

namespace py = pybind11;
using tam_sched::Engine;

namespace {

py::dict collect(Engine& e, long n);

py::dict run_py(Engine& e, py::array_t<double> submit, py::array_t<double> dur, py::array_t<int> gpus) {
  auto s = submit.unchecked<1>();
  auto d = dur.unchecked<1>();
  auto g = gpus.unchecked<1>();
  const long n = (long)s.shape(0);
  std::vector<double> sv(n), dv(n);
  std::vector<int> gv(n);
  for (long i = 0; i < n; ++i) { sv[i] = s(i); dv[i] = d(i); gv[i] = g(i); }
  e.run(sv.data(), dv.data(), gv.data(), n);
  return collect(e, n);
}

py::dict collect(Engine& e, long n) {
  py::array_t<double> st(n), en(n);
  py::array_t<int> pre(n), res(n), pro(n);
  auto ST = st.mutable_unchecked<1>();
  auto EN = en.mutable_unchecked<1>();
  auto PR = pre.mutable_unchecked<1>();
  auto RS = res.mutable_unchecked<1>();
  auto PM = pro.mutable_unchecked<1>();
  const auto& jobs = e.jobs();
  for (long i = 0; i < n; ++i) {
    ST(i) = jobs[i].start; EN(i) = jobs[i].end;
    PR(i) = jobs[i].preempt; RS(i) = jobs[i].resume; PM(i) = jobs[i].promote;
  }
  py::dict out;
  out["start"] = st; out["end"] = en; out["preempt"] = pre; out["resume"] = res;
  out["promote"] = pro; out["events"] = e.events();
  return out;
}

py::dict run_topo_py(Engine& e, py::array_t<double> submit, py::array_t<double> dur, py::array_t<int> gpus,
                     py::array_t<int> gpw, py::array_t<int> tcpu, py::array_t<int> tmem,
                     py::array_t<unsigned char> sens) {
  const long n = (long)submit.shape(0);
  if (dur.shape(0) != n || gpus.shape(0) != n || gpw.shape(0) != n || tcpu.shape(0) != n ||
      tmem.shape(0) != n || sens.shape(0) != n)
    throw std::invalid_argument("sched_core.run_topo: per-job arrays must have equal length");
  auto c = [](auto a) { return a.template unchecked<1>(); };
  auto s = c(submit); auto d = c(dur); auto g = c(gpus); auto w = c(gpw); auto cp = c(tcpu); auto mm = c(tmem);
  auto se = c(sens);
  std::vector<double> sv(n), dv(n);
  std::vector<int> gv(n), wv(n), cv(n), mv(n);
  std::vector<unsigned char> ev(n);
  for (long i = 0; i < n; ++i) {
    sv[i] = s(i); dv[i] = d(i); gv[i] = g(i); wv[i] = w(i); cv[i] = cp(i); mv[i] = mm(i); ev[i] = se(i);
  }
  e.run_topo(sv.data(), dv.data(), gv.data(), wv.data(), cv.data(), mv.data(), ev.data(), n);
  return collect(e, n);
}

void set_costs_py(Engine& e, bool net, double bw_mbps, double latency, int ckpt, double host_gbps,
                  double h2d_gbps, double xgmi_gbps, double budget_bytes, std::vector<double> ckpt_b,
                  std::vector<double> net_sd, std::vector<double> net_c, std::vector<double> net_bytes) {
  tam_sched::Costs c;
  c.net = net; c.bw_mbps = bw_mbps; c.latency = latency; c.ckpt = ckpt;
  c.host_gbps = host_gbps; c.h2d_gbps = h2d_gbps; c.xgmi_gbps = xgmi_gbps; c.budget = budget_bytes;
  if (ckpt < 0 || ckpt > 2) throw std::invalid_argument("sched_core.set_costs: ckpt must be 0, 1 or 2");
  e.set_costs(c, std::move(ckpt_b), std::move(net_sd), std::move(net_c), std::move(net_bytes));
}

py::dict costs_py(Engine& e) {
  const auto& jobs = e.jobs();
  const long n = (long)jobs.size();
  py::array_t<double> ov(n), by(n);
  auto O = ov.mutable_unchecked<1>();
  auto B = by.mutable_unchecked<1>();
  for (long i = 0; i < n; ++i) { O(i) = jobs[i].overhead; B(i) = jobs[i].ckpt_bytes; }
  py::dict out;
  out["overhead"] = ov; out["ckpt_bytes"] = by;
  return out;
}

}  // namespace

PYBIND11_MODULE(_sched_core, m) {
  m.doc() = "tiresias_amd native event-engine core (count / yarn / tiresias placement)";
  py::class_<Engine>(m, "Engine")
      .def(py::init<const std::string&, int, std::vector<double>, double, double, std::vector<double>, bool>(),
           py::arg("policy"), py::arg("total_gpus"), py::arg("queue_limits") = std::vector<double>{},
           py::arg("solve_starvation") = 0.0, py::arg("gittins_delta") = 3250.0,
           py::arg("prior") = std::vector<double>{}, py::arg("online_prior") = false)
      .def("run", &run_py, py::arg("submit"), py::arg("duration"), py::arg("gpus"))
      .def("set_topology", &Engine::set_topology, py::arg("placement"), py::arg("switches"),
           py::arg("nodes_per_switch"), py::arg("gpus_per_node"), py::arg("cpus"), py::arg("mem"))
      .def("set_costs", &set_costs_py, py::arg("network"), py::arg("bw_mbps"), py::arg("latency"),
           py::arg("ckpt"), py::arg("host_gbps"), py::arg("h2d_gbps"), py::arg("xgmi_gbps"),
           py::arg("budget_bytes"), py::arg("ckpt_bytes"), py::arg("net_slowdown"), py::arg("net_iter_s"),
           py::arg("net_bytes"))
      .def("costs", &costs_py)
      .def("set_spread_wait", &Engine::set_spread_wait, py::arg("on"))
      .def("set_spread_node", &Engine::set_spread_node, py::arg("on"))
      .def("set_spread_price", &Engine::set_spread_price, py::arg("on"))
      .def("set_lazy_preempt", &Engine::set_lazy_preempt, py::arg("on"))
      .def("spread_decisions", &Engine::spread_decisions, py::arg("spread"))
      .def("run_topo", &run_topo_py, py::arg("submit"), py::arg("duration"), py::arg("gpus"),
           py::arg("gpu_per_worker"), py::arg("cpu_per_task"), py::arg("mem_per_task"), py::arg("sensitive"));
}
