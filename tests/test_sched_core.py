"""The native event core must reproduce the Python engine job-for-job
(count placement), and be much faster on large traces."""
import time

import numpy as np
import pytest

from tiresias_amd.config import ClusterSpec, SimConfig
from tiresias_amd.engine import native
from tiresias_amd.engine.sim import Simulator
from tiresias_amd.trace.synth import philly_like_trace

pytestmark = pytest.mark.skipif(not native.available(), reason="native core not built")


def _cfg(policy, gpus=32):
    return SimConfig(schedule=policy, scheme="count", num_queue=3, queue_limits=[2000.0, 20000.0],
                     gittins_delta=1500.0, solve_starvation=2.0 if policy.startswith("dlas") else 0.0,
                     cluster=ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=gpus,
                                         num_cpu_p_node=100000, mem_p_node=100000))


@pytest.mark.parametrize("policy", list(native.SUPPORTED))
@pytest.mark.parametrize("seed", [0, 1])
def test_native_matches_python(policy, seed):
    specs = philly_like_trace(250, 32, load=1.4, seed=seed, median_duration=400)
    c = _cfg(policy)
    sim = Simulator(c, specs)
    ps = sim.run()
    ns = native.simulate_native(c, specs)
    py_end = np.array([sim.jobs[s.job_id].end_time for s in specs])
    py_pre = np.array([sim.jobs[s.job_id].preempt_count for s in specs])
    assert ns["finished"] == ps["finished"]
    np.testing.assert_allclose(ns["per_job"]["end"], py_end, rtol=1e-9, atol=1e-6)
    np.testing.assert_array_equal(ns["per_job"]["preempt"], py_pre)
    assert ns["avg_jct"] == pytest.approx(ps["avg_jct"], rel=1e-9)


def test_native_large_trace_fast():
    specs = philly_like_trace(20000, 512, load=1.1, seed=3, median_duration=900)
    t = time.perf_counter()
    s = native.simulate_native(_cfg("dlas-gpu", gpus=512), specs)
    assert s["finished"] == 20000
    assert time.perf_counter() - t < 60


def _topo_cfg(policy, scheme):
    # 2 racks x 4 nodes x 8 GPUs, reference-default task shape (12 CPU / 60 GB
    # per task): cross-node gangs, rack choice and fragmentation all matter
    return SimConfig(schedule=policy, scheme=scheme, num_queue=3, queue_limits=[2000.0, 20000.0],
                     gittins_delta=1500.0, solve_starvation=2.0 if policy.startswith("dlas") else 0.0,
                     cluster=ClusterSpec(num_switch=2, num_node_p_switch=4, num_gpu_p_node=8,
                                         num_cpu_p_node=128, mem_p_node=512))


@pytest.mark.parametrize("scheme", ["yarn", "tiresias"])
@pytest.mark.parametrize("policy", ["fifo", "shortest", "dlas-gpu", "gittins", "dlas-gpu-gittins"])
def test_native_topology_placement_matches_python(policy, scheme):
    """Native yarn / tiresias placement (racks x nodes x devices, per-node
    CPU / memory, skew-aware consolidation) reproduces the Python engine
    job-for-job on a 1000-job trace over 64 GPUs with 16/32-GPU gangs."""
    specs = philly_like_trace(1000, 64, load=1.3, seed=11, median_duration=500)
    c = _topo_cfg(policy, scheme)
    prior = sorted(s.duration * s.num_gpu for s in philly_like_trace(1000, 64, load=1.3, seed=99,
                                                                      median_duration=500))
    sim = Simulator(c, specs, prior=prior)
    ps = sim.run()
    ns = native.simulate_native(c, specs, prior=prior)
    py_end = np.array([sim.jobs[s.job_id].end_time for s in specs], dtype=float)
    py_pre = np.array([sim.jobs[s.job_id].preempt_count for s in specs])
    assert ns["finished"] == ps["finished"] == len(specs)
    np.testing.assert_allclose(ns["per_job"]["end"], py_end, rtol=1e-9, atol=1e-6)
    np.testing.assert_array_equal(ns["per_job"]["preempt"], py_pre)
    assert ns["scheme"] == scheme


@pytest.mark.parametrize("ckpt,net", [("host", False), ("measured", False), ("none", True), ("measured", True),
                                      ("hbm", True)])
@pytest.mark.parametrize("scheme,policy", [("yarn", "dlas-gpu"), ("tiresias", "gittins"),
                                           ("count", "dlas-gpu"), ("yarn", "fifo")])
def test_native_priced_matches_python(ckpt, net, scheme, policy, tmp_path):
    """PRICED replays (BASELINE config 1 with costs): checkpoint save /
    restore stalls (host path, HBM residency with xGMI moves, the measured
    MI355X bandwidth table) and the spread-gang network rate (measured
    slowdowns for the profiled models, analytic all-reduce for the rest)
    give the Python engine's per-job end times, preemption counts and
    checkpoint overheads."""
    specs = philly_like_trace(600, 64, load=1.3, seed=5, median_duration=500)
    c = _topo_cfg(policy, scheme)
    c.ckpt_policy = ckpt
    c.enable_network_costs = net
    c.ckpt_hbm_budget_gb = 2.0                 # small budget: both the resident and the host path
    # measured 2-node slowdowns for two families; every other model takes
    # the analytic all-reduce
    prof = tmp_path / "skew.json"
    prof.write_text('{"vgg16": {"slowdown": 1.7}, "resnet50": {"slowdown": 1.04}}')
    c.skew_profile = str(prof)
    prior = sorted(s.duration * s.num_gpu for s in philly_like_trace(600, 64, load=1.3, seed=98,
                                                                     median_duration=500))
    sim = Simulator(c, specs, prior=prior)
    ps = sim.run()
    ns = native.simulate_native(c, specs, prior=prior)
    assert ns["priced"]
    py_end = np.array([sim.jobs[s.job_id].end_time for s in specs], dtype=float)
    py_pre = np.array([sim.jobs[s.job_id].preempt_count for s in specs])
    py_ov = np.array([sim.jobs[s.job_id].overhead_time for s in specs], dtype=float)
    assert ns["finished"] == ps["finished"]
    np.testing.assert_array_equal(ns["per_job"]["preempt"], py_pre)
    np.testing.assert_allclose(ns["per_job"]["end"], py_end, rtol=1e-9, atol=1e-6)
    np.testing.assert_allclose(ns["per_job"]["overhead"], py_ov, rtol=1e-9, atol=1e-9)
    if ckpt != "none" and policy != "fifo":
        assert ns["ckpt_overhead_s"] > 0


def test_price_rule_native_equals_python():
    """spread_rule "price" (the wait-vs-spread penalty also charging the
    queued gangs the fragments delay, engine/spread.py::fragment_cost):
    the native core takes the same decisions as the Python engine on a
    priced Philly-shaped replay (terms summed in ascending order in both)."""
    import csv as _csv
    import dataclasses
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    import sweep_10k as S
    from tiresias_amd.engine.native import simulate_native
    from tiresias_amd.engine.sim import simulate

    hist = S._trace(600, 1.2, 7919)
    prior = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"prior_price_{os.getpid()}.csv")
    with open(prior, "w", newline="") as f:
        w = _csv.writer(f)
        w.writerow(["duration"])
        for x in hist:
            w.writerow([round(x.duration * x.num_gpu, 3)])
    try:
        specs = S._trace(600, 1.2, 0)
        for pol in ("gittins", "dlas-gpu"):
            cfg = dataclasses.replace(S._cfg(pol, "tiresias", prior, 0, "measured", True, "lazy"), spread_rule="price")
            nat, py = simulate_native(cfg, specs), simulate(cfg, specs)
            assert nat["finished"] == py["finished"] and nat["preemptions"] == py["preemptions"]
            assert abs(nat["avg_jct"] - py["avg_jct"]) < 1e-6 * py["avg_jct"]
    finally:
        os.remove(prior)
