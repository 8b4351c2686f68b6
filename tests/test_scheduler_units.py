"""Unit tests: flags, trace readers, cluster accounting, placement schemes,
policy orderings, Gittins index, k-means (SURVEY §4 test plan 1)."""
import csv
import math
import random

import pytest

from tiresias_amd.cluster.topology import Cluster, PlacementError
from tiresias_amd.config import ClusterSpec, SimConfig
from tiresias_amd.config import flags as fl
from tiresias_amd.core.job import Job, JobSpec, JobState
from tiresias_amd.placement import make_placement
from tiresias_amd.policy import make_policy, policies
from tiresias_amd.policy.horus import kmeans_jobs
from tiresias_amd.policy.las import GittinsTable
from tiresias_amd.trace import readers, synth


def spec(i, g=1, d=10.0, t=0.0, **kw):
    return JobSpec(job_id=str(i), submit_time=t, duration=d, num_gpu=g, **kw)


# ------------------------------------------------------------------ flags
def test_flags_parse_and_negation():
    F = fl._FlagValues()
    object.__setattr__(F, "_defs", {})
    F._define("schedule", "fifo", "", "str")
    F._define("pack", False, "", "bool")
    F._define("num_queue", 1, "", "int")
    F._define("queue_limits", [], "", "list")
    rest = F.parse(["--schedule", "dlas-gpu", "--pack", "--num_queue=3", "--queue_limits", "10,20",
                    "--unknown", "x"])
    assert F.schedule == "dlas-gpu" and F.pack is True and F.num_queue == 3
    assert F.queue_limits == ["10", "20"] and "--unknown" in rest
    F.parse(["--nopack"])
    assert F.pack is False
    F.parse(["--pack=f"])
    assert F.pack is False


def test_simconfig_from_flags(tmp_path):
    from tiresias_amd.config import FLAGS, define_flags

    define_flags()
    p = tmp_path / "spec.csv"
    p.write_text("num_switch,num_node_p_switch,num_gpu_p_node,num_cpu_p_node,mem_p_node\n1,16,4,128,254\n")
    FLAGS.parse(["--schedule", "dlas-gpu", "--cluster_spec", str(p), "--queue_limits", "100,200"])
    c = SimConfig.from_flags()
    assert c.schedule == "dlas-gpu" and c.queue_limits == [100.0, 200.0]
    assert c.cluster.num_node_p_switch == 16 and c.cluster.num_gpu_p_node == 4
    FLAGS.parse([])


# ------------------------------------------------------------------ traces
def test_live_trace_reader(tmp_path):
    p = tmp_path / "t.csv"
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["type", "normalized_time", "minutes", "gpu_per_container", "used_gpus",
                    "gpu_utilization_avg", "gpu_utilization_max", "memory_avg", "memory_max"])
        w.writerow(["noninteractive", 30000, 10, 1, 2, 50, 80, 2 ** 30, 2 ** 31])
        w.writerow(["interactive", 10000, 5, 1, 1, 50, 80, 2 ** 30, 2 ** 31])
        w.writerow(["noninteractive", 10000, 4, 2, 4, 40, 60, 2 ** 30, 2 ** 31])
        w.writerow(["noninteractive", 20000, "", 1, 1, 40, 60, 2 ** 30, 2 ** 31])
    assert readers.detect_schema(str(p)) == "live"
    s = readers.read_trace(str(p))
    assert [x.submit_time for x in s] == [0.0, 2.0]           # rebased, /10000, NaN dropped
    assert s[0].num_gpu == 4 and s[0].gpu_per_worker == 2 and s[0].duration == 4
    assert s[1].gpu_mem_max == pytest.approx(2048.0)           # bytes -> MiB


def test_tiresias_trace_roundtrip(tmp_path):
    specs = synth.SampleTraceGenerator(seed=1).generate_specs(20, max_gpu=16)
    p = tmp_path / "tr.csv"
    readers.write_tiresias_trace(str(p), specs)
    back = readers.read_trace(str(p))
    assert [(b.job_id, b.num_gpu, round(b.duration, 3)) for b in back] == \
           [(s.job_id, s.num_gpu, round(s.duration, 3)) for s in specs]


def test_streaming_reader():
    r = readers.StreamingReader([spec(i, t=float(i)) for i in range(5)])
    assert [s.job_id for s in r.release(1.5)] == ["0", "1"]
    assert r.next_time() == 2.0 and r.remaining() == 3
    assert [s.job_id for s in r.release(10)] == ["2", "3", "4"]
    assert r.next_time() == math.inf


def test_sample_generator_seeded_and_populations():
    a = synth.SampleTraceGenerator(seed=3).generate_trace(50)
    b = synth.SampleTraceGenerator(seed=3).generate_trace(50)
    assert a == b
    assert set(a["duration"]) <= set(synth.DURATION_SAMPLE)
    assert all(1 <= g < 128 for g in a["num_gpu"]) and all(20 <= i < 44 for i in a["interval"])


def test_philly_like_trace_shape():
    t = synth.philly_like_trace(2000, 64, load=1.0, seed=0)
    frac1 = sum(1 for s in t if s.num_gpu == 1) / len(t)
    assert 0.6 < frac1 < 0.8
    assert all(s.num_gpu <= 64 for s in t)
    assert all(t[i].submit_time <= t[i + 1].submit_time for i in range(len(t) - 1))
    assert {s.model for s in t} == {"resnet50", "vgg16", "transformer", "gnmt"}


# ------------------------------------------------------------------ cluster
def test_commit_release_conservation_d2():
    c = Cluster(ClusterSpec(num_switch=1, num_node_p_switch=2, num_gpu_p_node=4))
    j = Job(spec(0, g=3))
    alloc = c.commit(j, [("1", (0,)), ("1", (1,)), ("2", (0,))])
    assert alloc == {"1": [0, 1], "2": [0]}
    assert c.free_gpus() == 5
    c.check_invariants()
    j2 = Job(spec(1, g=2))
    with pytest.raises(PlacementError):
        c.commit(j2, [("1", (0,)), ("1", (2,))])    # device 0 busy -> nothing applied
    c.check_invariants()
    assert c.free_gpus() == 5
    c.release(j)
    c.check_invariants()
    assert c.free_gpus() == 8 and all(n.cpu_used == 0 for n in c.nodes.values())


def test_cpu_memory_limits_enforced():
    c = Cluster(ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=8, num_cpu_p_node=30,
                            mem_p_node=512))
    j = Job(spec(0, g=3))                            # 3 tasks x 12 cpu > 30
    assert make_placement("count").plan(c, j) is None


def test_virtual_nodes_partition():
    c = Cluster(ClusterSpec.mi355x_node(), virtual_nodes="2x4")
    assert len(c.nodes) == 2 and c.num_gpus == 8


# ------------------------------------------------------------------ placement
def _cluster(nodes=2, gpn=4, racks=1, pack=False):
    return Cluster(ClusterSpec(num_switch=racks, num_node_p_switch=nodes, num_gpu_p_node=gpn), pack=pack)


@pytest.mark.parametrize("scheme", ["count", "yarn", "random", "crandom", "greedy", "balance", "cbalance",
                                    "horus", "gandiva", "pack", "tiresias", "lp"])
def test_every_scheme_produces_valid_plans(scheme):
    c = _cluster(nodes=4, gpn=4, racks=2, pack=scheme in ("horus", "gandiva", "pack"))
    pl = make_placement(scheme, rng=random.Random(0))
    placed = 0
    for i, g in enumerate([1, 2, 4, 3, 1, 5, 2]):
        j = Job(spec(i, g=g, model="resnet50"))
        p = pl.plan(c, j)
        if p is not None:
            assert c.validate(j, p) is None
            c.commit(j, p)
            placed += 1
        c.check_invariants()
    assert placed >= 4


def test_yarn_consolidates_small_gangs():
    c = _cluster(nodes=2, gpn=4)
    pl = make_placement("yarn")
    a = Job(spec(0, g=3))
    c.commit(a, pl.plan(c, a))                      # node 1: 1 free
    b = Job(spec(1, g=2))
    p = pl.plan(c, b)
    assert {nid for nid, _ in p} == {"2"}           # never split a 2-GPU gang across nodes
    c.commit(b, p)
    d = Job(spec(2, g=3))
    assert pl.plan(c, d) is None                    # 3 free GPUs but on 2 nodes


def test_tiresias_skew_aware():
    c = _cluster(nodes=2, gpn=4)
    pl = make_placement("tiresias", sensitivity=lambda j: j.spec.model == "vgg16")
    a = Job(spec(0, g=3))
    c.commit(a, [("1", (0,)), ("1", (1,)), ("1", (2,))])   # node1: 1 free, node2: 4 free
    # insensitive job takes the fragment first (keeps node 2 whole)
    r = Job(spec(1, g=1, model="resnet50"))
    assert pl.plan(c, r)[0][0] == "1"
    # sensitive 2-GPU gang: consolidated on node 2
    v = Job(spec(2, g=2, model="vgg16"))
    assert {nid for nid, _ in pl.plan(c, v)} == {"2"}
    # sensitive gang bigger than any free node -> waits; insensitive may spread
    c.commit(Job(spec(9, g=1)), [("2", (0,))])
    big_v = Job(spec(3, g=4, model="vgg16"))
    big_r = Job(spec(4, g=4, model="resnet50"))
    assert pl.plan(c, big_v) is None
    assert pl.plan(c, big_r) is not None


def test_tiresias_node_rule_never_fragments_node_sized_gangs():
    """spread_rule "node" (default): with the wait-vs-spread advisor set, an
    insensitive gang that fits one node waits for a free node instead of
    taking fragments across nodes -- even when the advisor would spread it
    (rule "wait"); a gang wider than a node still consults the advisor
    (profiles/r5/spread_node_rule.md)."""
    class Always:
        decisions = {"spread": 0, "wait": 0}

        def should_spread(self, *a, **k):
            self.decisions["spread"] += 1
            return True

    c = _cluster(nodes=2, gpn=4)
    c.commit(Job(spec(8, g=2)), [("1", (0,)), ("1", (1,))])
    c.commit(Job(spec(9, g=2)), [("2", (0,)), ("2", (1,))])      # 2 free on each node
    r4 = Job(spec(1, g=4, model="resnet50"))
    pl = make_placement("tiresias", sensitivity=lambda j: False)
    pl.advisor, pl.jobs_by_id = Always(), {}
    pl.spread_node_gangs = True                                   # rule "wait"
    assert len({nid for nid, _ in pl.plan(c, r4)}) == 2
    pl.spread_node_gangs = False                                  # rule "node"
    assert pl.plan(c, r4) is None
    r2 = Job(spec(2, g=2, model="resnet50"))                      # fits one node: best-fit there
    assert len({nid for nid, _ in pl.plan(c, r2)}) == 1
    c8 = _cluster(nodes=3, gpn=4)
    c8.commit(Job(spec(7, g=2)), [("1", (0,)), ("1", (1,))])
    r8 = Job(spec(3, g=8, model="resnet50"))                      # wider than a node: fullest-free first
    assert sorted({nid for nid, _ in pl.plan(c8, r8)}) == ["2", "3"]
    pl.spread_node_gangs = True                                   # rule "wait": fragments first
    assert len({nid for nid, _ in pl.plan(c8, r8)}) == 3
    pl.spread_node_gangs = False
    c8.commit(Job(spec(6, g=1)), [("2", (0,))])                   # no 2 whole nodes left: the advisor decides
    n0 = Always.decisions["spread"]
    assert len({nid for nid, _ in pl.plan(c8, r8)}) == 3
    assert Always.decisions["spread"] == n0 + 1


def test_priced_node_rule_vs_wait_rule_and_yarn():
    """Priced replay (measured checkpoint stalls, spread gangs at the
    network-limited rate), lazy preemption, Gittins, 3000 Philly-shaped jobs
    on 64 GPUs, 3 seeds: the node rule (a node-sized gang never fragments, a
    wider one packs the fullest-free nodes) beats both yarn's
    consolidate-always placement (measured 0.93-0.97x) and the round-4 wait
    rule (1.11-1.19x yarn) on avg JCT on every seed; the native core matches
    the Python engine on the node-rule replay (profiles/r5/spread_node_rule.md)."""
    import dataclasses
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    import sweep_10k as S
    from tiresias_amd.engine.native import simulate_native
    from tiresias_amd.engine.sim import simulate

    ratios = []
    for seed in (0, 1, 2):
        hist = S._trace(3000, 1.2, seed + 7919)
        prior = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"prior_{os.getpid()}_{seed}.csv")
        with open(prior, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["duration"])
            for x in hist:
                w.writerow([round(x.duration * x.num_gpu, 3)])
        specs = S._trace(3000, 1.2, seed)
        jct = {}
        for scheme, rule in (("yarn", "node"), ("tiresias", "node"), ("tiresias", "wait")):
            cfg = dataclasses.replace(S._cfg("gittins", scheme, prior, seed, "measured", True, "lazy"),
                                      spread_rule=rule)
            r = simulate_native(cfg, specs)
            jct[(scheme, rule)] = r["avg_jct"]
            if seed == 0 and scheme == "tiresias" and rule == "node":
                py = simulate(cfg, specs)
                assert py["finished"] == r["finished"] and py["preemptions"] == r["preemptions"]
                assert abs(py["avg_jct"] - r["avg_jct"]) < 1e-6 * py["avg_jct"]
        os.remove(prior)
        assert jct[("tiresias", "node")] < jct[("tiresias", "wait")], (seed, jct)
        ratios.append(jct[("tiresias", "node")] / jct[("yarn", "node")])
    assert max(ratios) < 0.99, ratios


def test_horus_prefers_low_cost_and_colocates():
    c = _cluster(nodes=1, gpn=2, pack=True)
    pl = make_placement("horus")
    a = Job(spec(0, g=1, gpu_util_avg=90, gpu_util_max=95, gpu_mem_max=1000))
    c.commit(a, pl.plan(c, a))
    b = Job(spec(1, g=1, gpu_util_avg=10, gpu_util_max=20, gpu_mem_max=1000))
    p = pl.plan(c, b)
    assert p[0][1] != c.placed["0"][0][1]          # the idle device is cheaper
    c.commit(b, p)
    d = Job(spec(2, g=1, gpu_util_avg=10, gpu_util_max=20, gpu_mem_max=1000))
    assert pl.plan(c, d) is not None                # co-location allowed when packing


def test_lp_minimises_nodes():
    c = _cluster(nodes=3, gpn=4)
    c.commit(Job(spec(0, g=2)), [("1", (0,)), ("1", (1,))])
    pl = make_placement("lp")
    j = Job(spec(1, g=4))
    p = pl.plan(c, j)
    assert len({nid for nid, _ in p}) == 1


# ------------------------------------------------------------------ policies
def test_policy_registry_complete():
    want = {"fifo", "fjf", "sjf", "lpjf", "shortest", "shortest-gpu", "shortest-expected", "dlas",
            "dlas-gpu", "dlas-gpu-gittins", "gittins", "multi-dlas-gpu", "dlas-gpu-pack", "horus",
            "horus+", "gandiva"}
    assert want <= set(policies())


def test_gittins_index_hand_computed():
    # durations 1..10, delta 2: at a=0, P = #(S<=2)/10 = 0.2, E = mean(min(S,2)) = (1+2*9)/10 = 1.9
    t = GittinsTable(list(range(1, 11)), 2.0)
    assert t.index(0.0) == pytest.approx(0.2 / 1.9)
    # at a=5: alive = {6..10}; done = {6,7}; E = ((1+2) + 2*3)/5 = 1.8
    assert t.index(5.0) == pytest.approx((2 / 5) / 1.8)
    assert t.index(10.0) == 0.0
    # legacy (reference) formula: sum of raw durations
    tl = GittinsTable(list(range(1, 11)), 2.0, legacy_formula=True)
    assert tl.index(5.0) == pytest.approx(0.4 * 1e6 / ((6 + 7 + 2 * 3) / 5))


def test_horus_orders_by_utilisation():
    pol = make_policy("horus", SimConfig())
    jobs = [Job(spec(i, gpu_util_avg=u)) for i, u in enumerate([50, 10, 30])]
    for j in jobs:
        j.arrive(0)
    assert [j.job_id for j in pol.order(jobs, 0)] == ["1", "2", "0"]
    assert pol.lookahead == 5


def test_horus_plus_credits_and_kmeans_seeded():
    jobs = [Job(spec(i, g=g, gpu_util_avg=u)) for i, (g, u) in enumerate([(1, 10), (1, 12), (8, 90), (8, 95)])]
    import numpy as np
    _, a1, _ = kmeans_jobs(jobs, 2, np.random.RandomState(5))
    _, a2, _ = kmeans_jobs(jobs, 2, np.random.RandomState(5))
    assert a1 == a2 and a1[0] == a1[1] and a1[2] == a1[3] and a1[0] != a1[2]
    pol = make_policy("horus+", SimConfig(num_queue=2))
    for j in jobs:
        j.arrive(0)
    jobs[2].pending_time = jobs[3].pending_time = 50.0
    assert pol.order(jobs, 0)[0].job_id in ("2", "3")      # the big-credit queue goes first


def test_gandiva_time_slices_only_when_waiting():
    pol = make_policy("gandiva", SimConfig(timeslice=10.0))
    a, b = Job(spec(0)), Job(spec(1))
    a.arrive(0)
    a.start(0, {"1": [0]})
    a.extra["run_start"] = 0.0
    assert pol.preempt_now([a], 10.0) == []
    b.arrive(5)
    assert pol.next_event([a, b], 5.0) == 10.0
    assert pol.preempt_now([a, b], 10.0) == [a]


def test_multi_dlas_reserves_per_class():
    pol = make_policy("multi-dlas-gpu", SimConfig(num_queue=2, queue_limits=[100.0]))
    jobs = [Job(spec(i, g=g)) for i, g in enumerate([1, 1, 1, 4, 4])]
    for j in jobs:
        j.arrive(0)
        pol.on_arrival(j, 0)
    chosen = pol.select(pol.order(jobs, 0), 8, 0)
    assert sum(j.num_gpu for j in chosen) <= 8
    assert any(j.num_gpu == 4 for j in chosen) and any(j.num_gpu == 1 for j in chosen)


def test_tiresias_shares_only_when_full_and_picks_best_pair():
    """GPU sharing (pack) in the Tiresias placement: exclusive while a GPU is
    free; when full, a 1-GPU job joins the device whose 1-GPU occupant pairs
    best (lowest measured slowdown); never a gang's device; gangs never share."""
    c = Cluster(ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=3), pack=True,
                max_tasks_per_gpu=2)
    pl = make_placement("tiresias", pack=True)
    models = {"0": "vgg16", "1": "gnmt", "2": "resnet50"}
    pl.model_of = lambda jid: models[jid]
    slow = {("gnmt", "gnmt"): 1.38, ("gnmt", "vgg16"): 1.74, ("vgg16", "gnmt"): 1.74}
    pl.pair_cost = lambda a, b: slow.get((a, b), 1.6)
    kw = dict(gpu_mem_max=1000.0)
    a = Job(spec(0, g=1, model="vgg16", **kw))
    b = Job(spec(1, g=1, model="gnmt", **kw))
    for j in (a, b):
        p = pl.plan(c, j)
        assert c.device(*[(n, d[0]) for n, d in p][0]).is_idle()     # exclusive while free
        c.commit(j, p)
    g = Job(spec(2, g=1, model="resnet50", **kw))
    c.commit(g, pl.plan(c, g))
    assert c.free_gpus() == 0
    n = Job(spec(3, g=1, model="gnmt", **kw))
    p = pl.plan(c, n)
    assert p == [c.placed["1"][0]]                  # joins the gnmt device (1.38 < 1.74)
    gang = Job(spec(4, g=2, model="resnet50", **kw))
    assert pl.plan(c, gang) is None                 # gangs never share
    # an occupant that is part of a gang is never a sharing partner
    c2 = Cluster(ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=2), pack=True,
                 max_tasks_per_gpu=2)
    c2.commit(Job(spec(5, g=2, **kw)), [("1", (0,)), ("1", (1,))])
    assert pl.plan(c2, Job(spec(6, g=1, **kw))) is None


def test_sharing_yields_to_blocked_gang():
    """A gang that outranks the 1-GPU jobs sharing its GPUs preempts them
    (reason "unshare") instead of waiting behind lower-priority sharers."""
    from tiresias_amd.engine.sim import Simulator

    cfg = SimConfig(schedule="dlas-gpu", scheme="tiresias", num_queue=2, queue_limits=[2.0],
                    pack=True, max_tasks_per_gpu=2,
                    cluster=ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=2))
    jobs = [spec(i, g=1, d=40.0, t=0.0, model="resnet50", gpu_mem_max=1000.0) for i in range(4)]
    jobs.append(spec(9, g=2, d=5.0, t=5.0, model="resnet50", gpu_mem_max=1000.0))
    sim = Simulator(cfg, jobs)
    r = sim.run()
    assert r["finished"] == 5
    gang = sim.jobs["9"]
    # the 1-GPU jobs are demoted (2 GPU-s limit) long before t=5: the new gang
    # is top priority and starts on arrival although all 4 jobs were co-located
    assert gang.start_time == pytest.approx(5.0)


# ------------------------------------------------------------------ 2D-LAS queue order (reference run_sim.py:752-757, 837-847)
def _one_gpu(policy, **kw):
    return SimConfig(schedule=policy, scheme="count", num_queue=2, queue_limits=[10.0],
                     cluster=ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=1,
                                         num_cpu_p_node=100, mem_p_node=1000), **kw)


def test_dlas_demoted_job_queues_behind_pending():
    """A is demoted to Q1 (t=10) and preempted by B (t=15). When B is demoted
    at t=25 it joins the TAIL of Q1, behind the already-pending A: A runs."""
    from tiresias_amd.engine.sim import Simulator

    def at(t):
        sim = Simulator(_one_gpu("dlas"), [spec("A", d=100.0, t=0.0), spec("B", d=100.0, t=15.0)])
        sim.run(until=t)
        return sim.jobs["A"], sim.jobs["B"]

    a, b = at(20.0)
    assert b.is_running and a.is_pending and a.queue == 1
    a, b = at(26.0)
    assert a.is_running and b.is_pending and b.queue == 1


def test_last_pending_time_kept_until_promotion():
    """Starvation clock (reference :767-778): pending stretches since the job
    first ran accumulate across resumes; only a promotion clears them."""
    j = Job(spec("x", d=100.0))
    j.arrive(0.0)
    j.start(0.0, {"1": [0]})
    j.advance(5.0)
    j.preempt(5.0)
    j.advance(8.0)
    j.start(8.0, {"1": [0]})
    assert j.last_pending_time == pytest.approx(3.0)
    j.advance(9.0)
    j.preempt(9.0)
    j.advance(11.0)
    assert j.last_pending_time == pytest.approx(5.0)


def test_gittins_prior_never_sees_the_future():
    """Without a history file the Gittins table only holds FINISHED jobs'
    services (online); the replayed trace's own distribution needs an explicit
    opt-in and is flagged."""
    from tiresias_amd.engine.sim import Simulator

    specs = [spec(i, d=float(5 + 7 * i), t=float(i)) for i in range(6)]
    sim = Simulator(_one_gpu("gittins", gittins_delta=4.0), specs)
    assert sim.policy.table.data == []
    s = sim.run()
    assert s["prior"] == "online" and s["finished"] == 6
    got = sorted(sim.policy.table._samples)
    want = sorted(j.total_executed * j.num_gpu for j in sim.jobs.values())
    assert got == pytest.approx(want)
    oracle = Simulator(_one_gpu("gittins", gittins_delta=4.0, prior_mode="oracle"), specs)
    assert oracle.prior_source == "oracle" and len(oracle.policy.table.data) == 6


def test_gittins_prior_from_history_file(tmp_path):
    from tiresias_amd.engine.sim import Simulator

    p = tmp_path / "hist.csv"
    p.write_text("job_id,duration\n" + "".join(f"{i},{10 * (i + 1)}\n" for i in range(20)))
    sim = Simulator(_one_gpu("dlas-gpu-gittins", gittins_prior=str(p)), [spec(0, d=5.0)])
    sim.run()
    assert sim.prior_source == "file" and len(sim.policy.gittins.data) == 20


def test_lazy_preemption_skips_no_op_suspensions():
    """2 nodes x 4 GPUs, 2D-LAS + yarn: when B (4 GPUs, queue 0) arrives, the
    count prefix chooses it over the demoted V (3 GPUs), but no single node
    can take B even with V's GPUs free. The eager rule suspends V anyway and
    backfills it straight back (a no-op preemption that a priced or live run
    pays for); the lazy rule (default) leaves V running. Same schedule."""
    from tiresias_amd.config import ClusterSpec, SimConfig
    from tiresias_amd.core.job import JobSpec
    from tiresias_amd.engine.sim import Simulator

    def run(rule):
        specs = [JobSpec("F", 0.0, 1000.0, 1), JobSpec("V", 0.1, 1000.0, 3),
                 JobSpec("A", 50.0, 500.0, 3), JobSpec("B", 60.0, 100.0, 4)]
        cfg = SimConfig(schedule="dlas-gpu", scheme="yarn", num_queue=2, queue_limits=[60.0], preempt_rule=rule,
                        cluster=ClusterSpec(num_switch=1, num_node_p_switch=2, num_gpu_p_node=4))
        sim = Simulator(cfg, specs, check_invariants=True)
        sim.run()
        return {j.job_id: (j.start_time, j.end_time, j.preempt_count) for j in sim.jobs.values()}

    eager, lazy = run("eager"), run("lazy")
    assert eager["V"][2] == 1 and lazy["V"][2] == 0
    assert {k: v[:2] for k, v in eager.items()} == {k: v[:2] for k, v in lazy.items()}


def test_spread_rule_is_validated():
    """An unknown --spread_rule is an error in both engines, not a silent
    fallback to fragments-first."""
    import dataclasses
    from tiresias_amd.config import SimConfig
    from tiresias_amd.engine.native import simulate_native
    from tiresias_amd.engine.sim import simulate

    cfg = dataclasses.replace(SimConfig(schedule="dlas-gpu", scheme="tiresias"), spread_rule="nodes")
    specs = [spec(0, g=1)]
    with pytest.raises(ValueError, match="spread_rule"):
        simulate(cfg, specs)
    with pytest.raises(ValueError, match="spread_rule"):
        simulate_native(cfg, specs)
