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

py::dict run_py(Engine& e, py::array_t<double> submit, py::array_t<double> dur, py::array_t<int> gpus) {
  auto s = submit.unchecked<1>();
  auto d = dur.unchecked<1>();
  auto g = gpus.unchecked<1>();
  const long n = (long)s.shape(0);
  std::vector<double> sv(n), dv(n);
  std::vector<int> gv(n);
  for (long i = 0; i < n; ++i) { sv[i] = s(i); dv[i] = d(i); gv[i] = g(i); }
  e.run(sv.data(), dv.data(), gv.data(), n);
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

}  // namespace

PYBIND11_MODULE(_sched_core, m) {
  m.doc() = "tiresias_amd native event-engine core (count placement)";
  py::class_<Engine>(m, "Engine")
      .def(py::init<const std::string&, int, std::vector<double>, double, double, std::vector<double>, bool>(),
           py::arg("policy"), py::arg("total_gpus"), py::arg("queue_limits") = std::vector<double>{},
           py::arg("solve_starvation") = 0.0, py::arg("gittins_delta") = 3250.0,
           py::arg("prior") = std::vector<double>{}, py::arg("online_prior") = false)
      .def("run", &run_py, py::arg("submit"), py::arg("duration"), py::arg("gpus"));
}
