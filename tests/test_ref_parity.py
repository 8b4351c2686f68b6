"""Parity with an EXECUTION of the reference's live simulator.

``tests/fixtures/ref_parity.json`` was produced by ``tools/ref_parity.py``,
which runs the reference's ``run_sim.py`` (fixed-tick loop,
core/scheduling/schedule.py:178-212) in a scratch copy on two small
live-schema traces built so that none of the live-path defects (SURVEY.md §3
D1, D2, D8) changes the outcome, and records each job's start tick, end tick
and devices from the reference's own log.

``TickSimulator`` must reproduce every start and end tick for fifo/yarn,
horus/horus, gandiva/gandiva and horus+/horus+, and the exact devices for
fifo/yarn. horus+ re-clusters its queue with UNSEEDED k-means in the
reference (core/jobs/utils.py:36-67); the fixture run seeds numpy / random
in the launching interpreter (tools/ref_parity.py SEEDED) without touching
the reference's code, so its outcome is reproducible (on these traces the
queue never holds more than one job, so the clustering cannot reorder it).

A job's start is its placement COMMIT (``placed task`` at
core/scheduling/algorithm.py:170). Horus logs trial reservations for
placements that then fail -- the round-4 fixture took the first such trial
as the start, which made queued gangs look late in the reference. Among
equal-utilisation jobs the reference's heap (base_factory.py:2-14: ``<`` is
False on ties), not arrival order, picks the look-ahead; the tick engine's
horus / horus+ reproduce that heap operation for operation
(policy/horus.py ``ref_heap``), including horus+'s every-tick pop-all +
re-cluster (jobs_manager.py:115-140).

Two documented deviations are configured, not patched over:
  * the reference never applies its interference slowdown (D6,
    infra/node.py:201), so the sharing policies (horus, gandiva) are replayed
    with ``interference=0``;
  * horus/gandiva device choice is not pinned: the reference's scorer
    (core/scheduling/horus.py) picks different shared devices than ours; the
    timing still matches because co-location is free under D6.
"""
import json
import os

import pytest

from tiresias_amd.config import ClusterSpec, SimConfig
from tiresias_amd.core.job import JobSpec
from tiresias_amd.engine.sim import TickSimulator

FIXTURE = os.path.join(os.path.dirname(__file__), "fixtures", "ref_parity.json")
_FX = json.load(open(FIXTURE))
CASES = [(name, pair) for name, t in sorted(_FX["traces"].items()) for pair in sorted(t["results"])]


def _replay(trace: dict, pair: str) -> TickSimulator:
    schedule, scheme = pair.split("/")
    # reference job rows: (job_id, arrival tick, used_gpus, gpu_per_container, minutes);
    # it runs minutes * 0.5 ticks (schedule.py:187 gen_jobs(scale_factor=0.5))
    specs = [JobSpec(j[0], float(j[1]), j[4] * 0.5, j[2], gpu_per_worker=j[3]) for j in trace["jobs"]]
    cfg = SimConfig(schedule=schedule, scheme=scheme, engine="tick",
                    interference=0.0 if schedule != "fifo" else SimConfig.interference,
                    cluster=ClusterSpec(num_switch=1, num_node_p_switch=trace["nodes"],
                                        num_gpu_p_node=trace["gpus_per_node"]))
    sim = TickSimulator(cfg, specs)
    sim.run()
    return sim


def test_fixture_covers_all_pairs():
    assert len(CASES) == 10          # 2 traces x 4 pairs + the horus+ queue trace x 2
    for t in _FX["traces"].values():
        for res in t["results"].values():
            assert {j[0] for j in t["jobs"]} == set(res), "reference run did not finish every job"


@pytest.mark.parametrize("name,pair", CASES)
def test_tick_engine_matches_reference_execution(name, pair):
    trace = _FX["traces"][name]
    sim = _replay(trace, pair)
    want = {k: (float(v["start"]), float(v["end"])) for k, v in trace["results"][pair].items()}
    got = {j.job_id: (j.start_time, j.end_time) for j in sim.jobs.values()}
    assert got == want
    if pair == "fifo/yarn":
        for jid, v in trace["results"][pair].items():
            j = sim.jobs[jid]
            alloc = j.allocation or j.allocation_prev
            ours = sorted([node, d] for node, devs in alloc.items() for d in devs)
            assert ours == v["devices"], jid


def test_queued_gangs_divergence_is_not_the_reservation_leak():
    """Attribution of the round-4 horus / horus+ gap on the queued-gang trace:
    the reference run again with ONLY its reservation leak (SURVEY D2,
    infra/node.py:212-233) removed at run time (tools/ref_parity.py D2FIX)
    produces the same start / end ticks, so D2 does not change this trace's
    schedule; and the unpatched run does reserve devices for placements that
    then fail (the trial ticks the old fixture mistook for starts)."""
    t = _FX["traces"]["hplus_queue"]
    for pair, res in t["results"].items():
        fixed = t["results_d2fix"][pair]
        assert {k: (v["start"], v["end"]) for k, v in res.items()} == \
            {k: (v["start"], v["end"]) for k, v in fixed.items()}, pair
        trials = {k: v["trial_ticks"] for k, v in res.items() if v.get("trial_ticks")}
        assert trials, pair
        for k, ticks in trials.items():
            assert all(x < res[k]["start"] for x in ticks), (pair, k)


def test_tie_order_follows_the_reference_heap():
    """Equal-utilisation queued jobs: the event engine keeps arrival order,
    the tick engine the reference's heap order -- which on this trace starts
    job 5 before job 4 (both queued at tick 7), as the reference did."""
    t = _FX["traces"]["hplus_queue"]
    sim = _replay(t, "horus/horus")
    assert sim.jobs["5"].start_time < sim.jobs["4"].start_time
    ref = t["results"]["horus/horus"]
    assert ref["5"]["start"] < ref["4"]["start"]


@pytest.mark.parametrize("ci", range(len(_FX.get("kmeans", []))))
def test_kmeans_matches_reference(ci):
    """horus+ k-means against the reference's own ``clusterize`` EXECUTED on
    heterogeneous job features with numpy seeded per case
    (tools/ref_parity.py KM_SCRIPT; core/jobs/utils.py:14-67): init drawn
    with replacement, L1 assignment with first-minimum ties, centroids
    re-picked by the scalar feature-sum closest to the int-truncated mean
    (first minimum), random re-draw of empty clusters -- the same
    RandomState seed gives the same centroids, assignment and loss
    (VERDICT r5 item 7). Trace-level parity on such queues is out of reach:
    the reference's placement scorer and per-tick log draw from the same
    unseeded stream (tools/ref_parity.py)."""
    import numpy as np

    from tiresias_amd.core.job import Job
    from tiresias_amd.policy.horus import kmeans_jobs

    c = _FX["kmeans"][ci]
    jobs = []
    for i, f in enumerate(c["feats"]):
        workers, ua, gpw, gpus, um, ma, mm = f
        j = Job(JobSpec(str(i), 0.0, 1.0, int(gpus), gpu_per_worker=int(gpw), gpu_util_avg=ua, gpu_util_max=um,
                        gpu_mem_avg=ma, gpu_mem_max=mm))
        assert len(j.tasks) == workers
        jobs.append(j)
    cent, assign, loss = kmeans_jobs(jobs, c["k"], np.random.RandomState(c["seed"]))
    ref = c["reference"]
    assert cent == ref["cent"] and assign == ref["assign"]
    assert loss == pytest.approx(ref["loss"], rel=1e-9)
