"""Golden simulations with hand-derived JCTs (SURVEY §4 test plan 2) and the
reference defects the new engine must NOT reproduce (D1, D2, D8, D10)."""
import pytest

from tiresias_amd.config import ClusterSpec, SimConfig
from tiresias_amd.core.job import JobSpec
from tiresias_amd.engine.sim import Simulator, simulate
from tiresias_amd.metrics.logger import MetricsLogger


def cfg(schedule, scheme="count", gpus=4, nodes=1, **kw):
    return SimConfig(schedule=schedule, scheme=scheme,
                     cluster=ClusterSpec(num_switch=1, num_node_p_switch=nodes, num_gpu_p_node=gpus), **kw)


def J(i, t, g, d, **kw):
    return JobSpec(job_id=str(i), submit_time=t, num_gpu=g, duration=d, **kw)


def jcts(c, specs):
    sim = Simulator(c, specs, check_invariants=True)
    sim.run()
    return {j.job_id: round(j.jct, 6) for j in sim.jobs.values()}, sim


def test_fifo_head_of_line():
    out, _ = jcts(cfg("fifo"), [J(0, 0, 4, 10), J(1, 1, 2, 5), J(2, 2, 2, 5)])
    assert out == {"0": 10, "1": 14, "2": 13}


def test_fifo_blocks_but_fjf_backfills():
    specs = [J(0, 0, 3, 10), J(1, 1, 4, 2), J(2, 2, 1, 2)]
    out, _ = jcts(cfg("fifo"), specs)
    assert out == {"0": 10, "1": 11, "2": 12}      # job 2 waits behind job 1
    out, _ = jcts(cfg("fjf"), specs)
    assert out["2"] == 2                          # fit-job-first back-fills it


def test_dlas_gpu_demotion_and_preemption():
    # A (4 GPUs) crosses the 20 GPU-s threshold at t=5 -> Q1; B arrives at 6 in Q0 and preempts A
    c = cfg("dlas-gpu", queue_limits=[20.0])
    out, sim = jcts(c, [J(0, 0, 4, 20), J(1, 6, 4, 3)])
    assert out == {"0": 23, "1": 3}
    a = sim.jobs["0"]
    assert a.preempt_count == 1 and a.queue == 1


def test_dlas_time_vs_gpu_time():
    # dlas (time) demotes the 4-GPU job later than dlas-gpu
    specs = [J(0, 0, 4, 20), J(1, 6, 1, 3)]
    out_t, sim_t = jcts(cfg("dlas", queue_limits=[10.0]), specs)
    out_g, sim_g = jcts(cfg("dlas-gpu", queue_limits=[10.0]), specs)
    # dlas: A (4 GPUs) stays in Q0 until executed >= 10 s, so B waits until t=10
    assert out_t == {"0": 23, "1": 7}
    # dlas-gpu: A crosses 10 GPU-s at t=2.5, so B (arriving at 6) preempts it at once
    assert out_g == {"0": 23, "1": 3}
    assert sim_t.jobs["0"].preempt_count == 1 and sim_g.jobs["0"].preempt_count == 1


def test_srtf_preempts_longer_job():
    out, _ = jcts(cfg("shortest"), [J(0, 0, 4, 10), J(1, 2, 4, 3)])
    assert out == {"0": 13, "1": 3}


def test_sjf_orders_by_gpu_demand():
    out, _ = jcts(cfg("sjf"), [J(0, 0, 4, 10), J(1, 1, 2, 10), J(2, 1, 4, 1)])
    assert out == {"1": 10, "0": 20, "2": 20}


def test_starvation_promotion():
    # a long job demoted to Q1 and then starved is promoted back to Q0 with its
    # executed time reset (reference run_sim.py:771-778)
    from tiresias_amd.core.job import Job
    from tiresias_amd.policy import make_policy

    pol = make_policy("dlas-gpu", cfg("dlas-gpu", queue_limits=[8.0], solve_starvation=2.0))
    L = Job(J(0, 0, 4, 100))
    L.arrive(0.0)
    pol.on_arrival(L, 0.0)
    L.start(0.0, {"1": [0, 1, 2, 3]})
    L.advance(3.0)
    pol.update([L], 3.0)
    assert L.queue == 1                       # 12 GPU-s >= 8
    L.preempt(3.0)
    L.advance(8.9)
    pol.update([L], 8.9)
    assert L.queue == 1 and L.promote_count == 0      # 5.9 < 3 * 2
    assert pol.next_event([L], 8.9) == pytest.approx(9.0)
    L.advance(9.0)
    pol.update([L], 9.0)
    assert L.queue == 0 and L.promote_count == 1 and L.executed == 0.0
    # integration: promotions happen under a stream of short jobs
    specs = [J(0, 0, 4, 100)] + [J(i, 10 + 4 * (i - 1), 4, 4) for i in range(1, 40)]
    _, s_yes = jcts(cfg("dlas-gpu", queue_limits=[8.0], solve_starvation=2.0), specs)
    _, s_no = jcts(cfg("dlas-gpu", queue_limits=[8.0]), specs)
    assert s_yes.jobs["0"].promote_count > 0 and s_no.jobs["0"].promote_count == 0


def test_all_jobs_finish_even_when_queue_nonempty_d1():
    # reference D1: the loop stopped with queued jobs; ours drains everything
    specs = [J(i, 0.0, 4, 5) for i in range(10)]
    s = simulate(cfg("fifo"), specs)
    assert s["finished"] == 10 and s["makespan"] == pytest.approx(50)


def test_fifo_is_arrival_order_d8():
    specs = [J(0, 0, 4, 5), J(1, 1, 4, 5), J(2, 2, 4, 5)]
    out, sim = jcts(cfg("fifo"), specs)
    starts = sorted(sim.jobs.values(), key=lambda j: j.start_time)
    assert [j.job_id for j in starts] == ["0", "1", "2"]


def test_unplaceable_job_fails_not_hangs():
    s = simulate(cfg("dlas-gpu"), [J(0, 0, 8, 5), J(1, 0, 2, 5)])
    assert s["failed"] == 1 and s["finished"] == 1


def test_determinism_d10(tmp_path):
    from tiresias_amd.trace.synth import philly_like_trace

    specs = philly_like_trace(120, 32, load=1.3, seed=7)
    outs = []
    for k in range(2):
        d = tmp_path / f"run{k}"
        simulate(SimConfig(schedule="horus+", scheme="horus", num_queue=3, seed=3,
                           cluster=ClusterSpec(num_switch=1, num_node_p_switch=4, num_gpu_p_node=8)),
                 specs, out_dir=str(d))
        outs.append((d / "job.csv").read_text() + (d / "cluster.csv").read_text())
    assert outs[0] == outs[1]


def test_ckpt_costs_are_charged():
    specs = [J(0, 0, 4, 20, model="vgg16"), J(1, 6, 4, 3, model="vgg16")]
    free, _ = jcts(cfg("dlas-gpu", queue_limits=[20.0]), specs)
    paid, sim = jcts(cfg("dlas-gpu", queue_limits=[20.0], ckpt_policy="host", ckpt_bw_gbps=1.0), specs)
    assert paid["0"] > free["0"]
    assert sim.jobs["0"].ckpt_bytes > 0
    hbm, _ = jcts(cfg("dlas-gpu", queue_limits=[20.0], ckpt_policy="hbm"), specs)
    assert hbm["0"] == free["0"]        # resumed on the same GPUs: pointer swap


def test_outputs_written(tmp_path):
    from tiresias_amd.metrics.logger import CLUSTER_HEADER, JOB_HEADER
    import csv
    import json

    simulate(cfg("dlas-gpu"), [J(0, 0, 2, 5), J(1, 1, 2, 3)], out_dir=str(tmp_path))
    rows = list(csv.reader(open(tmp_path / "job.csv")))
    assert rows[0] == JOB_HEADER and len(rows) == 3
    crow = list(csv.reader(open(tmp_path / "cluster.csv")))
    assert crow[0] == CLUSTER_HEADER and len(crow) > 1
    for name in ("gpu", "cpu", "memory", "network"):
        assert (tmp_path / f"{name}.csv").exists()
    assert len(list(csv.reader(open(tmp_path / "gpu.csv")))) > 1
    s = json.load(open(tmp_path / "summary.json"))
    assert s["finished"] == 2 and s["avg_jct"] > 0
    assert (tmp_path / "decisions.jsonl").read_text().count('"finish"') == 2


def test_tick_engine_live_fifo_hand_derived():
    """The live reference's tick loop (core/scheduling/schedule.py:178-212),
    derived by reading it: at tick d arrivals with submit <= d are queued, at
    most ONE job is placed (FIFO head only, schedule_fifo: head-of-line
    blocking), then d += 1, every running job's processed time += 1
    (jobs_manager.py:143-147, job.py:53-56) and jobs with processed >=
    duration are released at tick d (jobs_manager.py:240-246). So a job placed
    at tick s ends at s + ceil(duration). Trace on one 4-GPU node:
      A t=0 2 GPU dur 2.5 -> placed 0, ends 3
      B t=0 1 GPU dur 3   -> placed 1 (one placement per tick), ends 4
      C t=0 4 GPU dur 1   -> blocked at 2, 3 (3 free after A), placed 4, ends 5
      D t=1 1 GPU dur 1   -> behind C (FIFO), placed 5, ends 6
    (Parity with an EXECUTION of the reference on larger traces is pinned in
    tests/test_ref_parity.py, fixture from tools/ref_parity.py.)"""
    from tiresias_amd.engine.sim import TickSimulator

    c = SimConfig(schedule="fifo", scheme="yarn", engine="tick",
                  cluster=ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=4))
    specs = [J("A", 0.0, 2, 2.5), J("B", 0.0, 1, 3.0), J("C", 0.0, 4, 1.0), J("D", 1.0, 1, 1.0)]
    sim = TickSimulator(c, specs)
    sim.run()
    got = {j.job_id: (j.start_time, j.end_time) for j in sim.jobs.values()}
    assert got == {"A": (0.0, 3.0), "B": (1.0, 4.0), "C": (4.0, 5.0), "D": (5.0, 6.0)}
