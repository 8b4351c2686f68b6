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


# Known gap (round 4): with SEVERAL whole-node jobs queued behind horus's
# packed GPUs, the reference runs queued jobs later and longer than ours (e.g.
# job 4: reference ticks 10-15 under horus, 13-16 under horus+; ours 7-10).
# The k-means side is pinned (every queued job has the same features, so both
# implementations cluster them identically); the divergence is in horus's
# packing / re-placement of queued gangs, not yet reproduced. Kept as a
# strict xfail so a fix shows up.
_UNPINNED = {("hplus_queue", "horus/horus"), ("hplus_queue", "horus+/horus+")}


@pytest.mark.parametrize("name,pair", [pytest.param(n, p, marks=pytest.mark.xfail(
    strict=True, reason="horus packing with several queued gangs: parity unpinned")) if (n, p) in _UNPINNED
    else (n, p) for n, p in CASES])
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
