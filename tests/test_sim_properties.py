"""Property tests (hypothesis): for random traces and every policy, all jobs
finish, JCT >= service time, GPU capacity is never exceeded and resources are
conserved after every event, no job starts before it is submitted."""
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from tiresias_amd.config import ClusterSpec, SimConfig
from tiresias_amd.core.job import JobSpec
from tiresias_amd.engine.sim import Simulator

POLICIES = ["fifo", "fjf", "sjf", "lpjf", "shortest", "shortest-gpu", "shortest-expected", "dlas",
            "dlas-gpu", "dlas-gpu-gittins", "gittins", "multi-dlas-gpu", "dlas-gpu-pack", "horus", "horus+",
            "gandiva"]

job_st = st.tuples(st.floats(0, 200, allow_nan=False), st.sampled_from([1, 1, 1, 2, 4, 8]),
                   st.floats(0.5, 300, allow_nan=False))


@pytest.mark.parametrize("policy", POLICIES)
@settings(max_examples=12, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(jobs=st.lists(job_st, min_size=1, max_size=25))
def test_policy_properties(policy, jobs):
    specs = [JobSpec(job_id=str(i), submit_time=round(t, 3), num_gpu=g, duration=round(d, 3),
                     gpu_util_avg=30.0, gpu_util_max=60.0, gpu_mem_max=2000.0)
             for i, (t, g, d) in enumerate(jobs)]
    cfg = SimConfig(schedule=policy, scheme="default", num_queue=2, queue_limits=[50.0],
                    solve_starvation=1.5, timeslice=20.0, replan_interval=60.0,
                    cluster=ClusterSpec(num_switch=1, num_node_p_switch=2, num_gpu_p_node=8))
    sim = Simulator(cfg, specs, check_invariants=True)
    sim.run(max_events=200000)
    for j in sim.jobs.values():
        assert j.end_time is not None, f"{policy}: job {j.job_id} never finished"
        assert j.start_time >= j.spec.submit_time - 1e-9
        # co-located (packing) jobs run slower, never faster than their service time
        assert j.jct >= j.spec.duration - 1e-6
        assert j.progress == pytest.approx(j.spec.duration)
    assert not sim.cluster.placed


@pytest.mark.parametrize("policy", ["dlas-gpu", "gittins", "fifo"])
@settings(max_examples=12, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(jobs=st.lists(job_st, min_size=1, max_size=25))
def test_tiresias_sharing_properties(policy, jobs):
    """Tiresias placement with GPU sharing when full (the bench's headline
    config): every job finishes, invariants hold after every event, no GPU
    holds more than 2 jobs, and gangs are never co-located."""
    specs = [JobSpec(job_id=str(i), submit_time=round(t, 3), num_gpu=g, duration=round(d, 3),
                     model=("resnet50", "vgg16", "transformer", "gnmt")[i % 4],
                     gpu_util_avg=30.0, gpu_util_max=60.0, gpu_mem_max=2000.0)
             for i, (t, g, d) in enumerate(jobs)]
    cfg = SimConfig(schedule=policy, scheme="tiresias", num_queue=2, queue_limits=[50.0], pack=True,
                    max_tasks_per_gpu=2, interference=0.5,
                    cluster=ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=8))
    sim = Simulator(cfg, specs, check_invariants=True)
    orig = sim.cluster.commit

    def commit(job, plan):
        alloc = orig(job, plan)
        for n in sim.cluster.nodes.values():
            for d in n.devices:
                assert len(d.tasks) <= 2
                if len(d.tasks) > 1:
                    assert all(sim.jobs[t.job_id].num_gpu == 1 for t in d.tasks.values())
        return alloc

    sim.cluster.commit = commit
    sim.run(max_events=200000)
    for j in sim.jobs.values():
        assert j.end_time is not None, f"{policy}: job {j.job_id} never finished"
        assert j.jct >= j.spec.duration - 1e-6
    assert not sim.cluster.placed
