// tiresias_amd — native discrete-event core for full-trace replays.
//
// The Python engine (tiresias_amd/engine/sim.py) models everything (topology
// placements, packing, interference, network, checkpoints, live runtime);
// it is O(active jobs) Python per event. Replaying the month-long NSDI'19
// trace (~10^5 jobs) across a policy sweep needs a native loop. This core
// implements the same event semantics for the resource-counting placement
// ("count") with the preemptive / non-preemptive policy family Tiresias is
// evaluated on — fifo, fjf, sjf, shortest, shortest-gpu, dlas, dlas-gpu,
// dlas-gpu-gittins, gittins — and is cross-checked job-for-job against the
// Python engine in tests/test_sched_core.py.
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
      .def("run_topo", &run_topo_py, py::arg("submit"), py::arg("duration"), py::arg("gpus"),
           py::arg("gpu_per_worker"), py::arg("cpu_per_task"), py::arg("mem_per_task"), py::arg("sensitive"));
}
