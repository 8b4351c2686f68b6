"""Fake (virtual-time) executor backend (SURVEY §4 plan item 4): the live
controller's scheduling, preemption and state-move protocol at world 8
without GPUs or processes, protocol-violation detection, spread-gang
penalties under virtual nodes, and the ``--backend fake`` CLI."""
import dataclasses

import pytest

import bench
from tiresias_amd.executor.fake import FakeCluster, ProtocolError, VirtualClock, run_fake


def _cfg(policy="dlas-gpu", scheme="tiresias", n=8, **kw):
    c = bench.make_cfg(policy, scheme, n, 3, "none", [0.05, 0.25, 1.0], False)
    return dataclasses.replace(c, **kw)


@pytest.mark.parametrize("policy,scheme", [("dlas-gpu", "tiresias"), ("fifo", "yarn"), ("gittins", "tiresias"),
                                           ("dlas-gpu-gittins", "random"), ("sjf", "count")])
def test_live_controller_world8_virtual_time(policy, scheme):
    jobs = bench.bench_trace(8, 24, 11, work_s=3.0)
    assert any(j.spec.num_gpu >= 4 for j in jobs)
    s = run_fake(_cfg(policy, scheme), jobs, 8, quantum=0.02,
                 prior=bench.history_prior(bench.bench_trace(8, 24, 99, work_s=3.0)))
    assert s["finished"] == len(jobs) and s["failed"] == 0
    assert s["backend"] == "fake" and s["virtual_s"] >= 3.0 * 0.9
    if policy != "fifo":
        assert s["preemptions"] > 0


def test_fake_tiresias_beats_fifo_like_the_simulator():
    jobs = bench.bench_trace(8, 24, 5, work_s=3.0)
    t = run_fake(_cfg(), jobs, 8, quantum=0.02)
    f = run_fake(_cfg("fifo", "yarn"), jobs, 8, quantum=0.02)
    assert t["avg_jct"] < f["avg_jct"]


def test_host_spill_and_p2p_moves_are_exercised():
    jobs = bench.bench_trace(8, 16, 21, work_s=2.0)
    s = run_fake(_cfg(ckpt_policy="host"), jobs, 8, quantum=0.02)
    st = s["fake_stats"]
    assert s["finished"] == len(jobs)
    assert st["spill_bytes"] > 0 and st["restore_bytes"] > 0
    s2 = run_fake(_cfg(), jobs, 8, quantum=0.02)
    assert s2["fake_stats"]["resident_resumes"] > 0


def test_spread_gangs_pay_under_virtual_nodes():
    """VGG-16 4-GPU gangs on 2x4 virtual nodes: random placement spreads
    some of them over the emulated link; skew-aware consolidation does not."""
    jobs = bench.scenario_trace("skew", 8, 2019)
    for j in jobs:
        j.model = "vgg16"
        j.spec.model = "vgg16"
        j.spec.num_gpu = 4
    base = dict(virtual_nodes="2x4", nic_gbps=12.5)
    t = run_fake(_cfg("dlas-gpu", "tiresias", **base), jobs, 8, quantum=0.05)
    r = run_fake(_cfg("dlas-gpu", "random", **base), jobs, 8, quantum=0.05)
    assert t["finished"] == r["finished"] == len(jobs)
    assert t["avg_jct"] < r["avg_jct"]


def _plan(actions, assign=None, deadline=None):
    return {"actions": actions, "assign": assign or {}, "deadline": deadline}


def test_protocol_violations_are_caught():
    fc = FakeCluster(4)
    st = {"op": "start", "job": "1", "model": "resnet50", "batch": None, "seed": 1}
    with pytest.raises(ProtocolError, match="without a communicator"):
        fc.apply(_plan([dict(st, ranks=(0, 1), source="fresh")]))
    fc = FakeCluster(4)
    fc.apply(_plan([dict(st, ranks=(0,), source="fresh")]))
    with pytest.raises(ProtocolError, match="resident resume"):
        fc.apply(_plan([dict(st, ranks=(1,), source="resident")]))
    with pytest.raises(ProtocolError, match="p2p move"):
        fc.apply(_plan([dict(st, ranks=(2,), source="p2p", donors={2: 3}, old=(3,))]))
    with pytest.raises(ProtocolError, match="does not hold"):
        fc.run(_plan([], {2: [("1", 3)]}), 0.0, {})
    with pytest.raises(ProtocolError, match="not resident"):
        fc.apply(_plan([{"op": "spill", "job": "9", "ranks": (0,)}]))
    with pytest.raises(ProtocolError, match="no rank holds"):
        fc.apply(_plan([{"op": "drop", "job": "9", "ranks": (0,)}]))
    fc.apply(_plan([{"op": "group", "ranks": (2, 3)}, dict(st, job="2", ranks=(2, 3), source="fresh")]))
    with pytest.raises(ProtocolError, match="different step counts"):
        fc.run(_plan([], {2: [("2", 3)], 3: [("2", 4)]}), 0.0, {})
    fc.apply(_plan([dict(st, job="3", ranks=(1,), source="fresh")]))
    with pytest.raises(ProtocolError, match="shares rank"):
        fc.run(_plan([], {2: [("2", 3), ("3", 1)], 3: [("2", 3)]}), 0.0, {})


def test_virtual_clock():
    c = VirtualClock()
    c.advance(1.5)
    assert c() == 1.5
    with pytest.raises(ValueError):
        c.advance(-1)


def test_backend_fake_cli(tmp_path):
    from tiresias_amd.cli import run_sim
    from tiresias_amd.core.job import JobSpec
    from tiresias_amd.trace.readers import write_tiresias_trace

    tr = tmp_path / "t.csv"
    write_tiresias_trace(str(tr), [JobSpec(str(i), 10.0 * i, 60.0 + 30 * i, 1 + (i % 3), model="resnet50")
                                   for i in range(12)])
    s = run_sim.main(["--backend", "fake", "--trace_file", str(tr), "--time_scale", "0.01",
                      "--schedule", "dlas-gpu", "--scheme", "tiresias", "--num_queue", "2",
                      "--queue_limits", "0.5", "--num_gpu_p_node", "8", "--log_path", str(tmp_path / "f"),
                      "--quantum", "0.05"])
    assert s["backend"] == "fake" and s["finished"] == 12
    assert (tmp_path / "f" / "job.csv").exists()


def test_fill_mode_keeps_barrier_idle_low_at_world8():
    """Bulk-synchronous rounds with fill mode (ranks keep stepping their job
    until the next plan) and finishing rounds (a round in which a job ends
    gives every other single-job rank a share of 0 steps, so the freed GPU
    is re-planned as soon as its job is done): on the headline trace at
    N = 8 the barrier idle stays under 3 % of GPU time, and each mechanism
    lowers it (executor/fake.py barrier accounting)."""
    def idle(fill, fill_rounds):
        jobs = bench.bench_trace(8, 24, 5)
        fc = FakeCluster(8, iter_s=dict(bench.TRACE_ITER_S), fill=fill)
        s = run_fake(_cfg(), jobs, 8, quantum=0.01, iter_s=dict(bench.TRACE_ITER_S), fake=fc,
                     prior=bench.history_prior(bench.bench_trace(8, 24, 5 + bench.HISTORY_SEED_OFFSET)),
                     fill_rounds=fill_rounds)
        st = s["fake_stats"]
        assert s["finished"] == len(jobs)
        # fill-mode accounting never runs a job past its iteration count: the
        # carry (steps in flight when the plan came) caps the next share and
        # fill
        assert s["overrun_iters"] <= 0, s["overrun_iters"]
        return st["barrier_idle_s"] / (st["barrier_idle_s"] + st["busy_s"])

    off, fill, both = idle(False, False), idle(True, False), idle(True, True)
    assert off > fill > both, (off, fill, both)
    assert both < 0.03, both
