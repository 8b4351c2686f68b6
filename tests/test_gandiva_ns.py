"""Legacy Gandiva node-set engine (reference run_sim.py:101-158,
infra/cluster.py:150-489): placement classes, time-slicing, grow/shrink."""
import pytest

from tiresias_amd.config import ClusterSpec, SimConfig
from tiresias_amd.core.job import JobSpec
from tiresias_amd.engine.sim import simulate
from tiresias_amd.trace.synth import philly_like_trace


def _cfg(nodes=1, gpn=4, **kw):
    return SimConfig(schedule="gandiva-ns", cluster=ClusterSpec(num_switch=1, num_node_p_switch=nodes,
                                                                num_gpu_p_node=gpn), **kw)


def test_timeslicing_oversubscribed_set():
    # 6 one-GPU jobs on one 4-GPU node: 4 run concurrently, the rest are
    # time-sliced in every 60 s; total work 6*120 GPU-s over 4 GPUs
    specs = [JobSpec(str(i), 0.0, 120.0, 1) for i in range(6)]
    s = simulate(_cfg(), specs)
    assert s["finished"] == 6
    assert s["preemptions"] > 0
    assert s["makespan"] >= 6 * 120 / 4 - 1e-6
    assert s["makespan"] <= 6 * 120 / 4 + 60 + 1e-6
    assert s["avg_jct"] >= 120


def test_node_sets_per_class_and_exact_finish():
    # 1-, 2- and 4-GPU jobs on 4 nodes x 4 GPUs: every class gets its own set
    specs = [JobSpec("a", 0.0, 35.0, 1), JobSpec("b", 0.0, 47.0, 2), JobSpec("c", 0.0, 61.0, 4),
             JobSpec("d", 5.0, 20.0, 8)]
    s = simulate(_cfg(nodes=4), specs)
    assert s["finished"] == 4
    assert s["preemptions"] == 0
    # exact (not tick-rounded) completion times; "d" (2 nodes) pends until
    # "a"'s one-node set is released at t=35, then runs 20 s -> JCT 50
    assert s["avg_jct"] == pytest.approx((35 + 47 + 61 + 50) / 4)


def test_too_big_job_fails_not_hangs():
    specs = [JobSpec("x", 0.0, 10.0, 64), JobSpec("y", 0.0, 10.0, 1)]
    s = simulate(_cfg(nodes=1), specs)
    assert s["finished"] == 1 and s["failed"] == 1


@pytest.mark.parametrize("mem", ["one", "legacy"])
def test_trace_completes_with_grow_shrink(tmp_path, mem):
    specs = philly_like_trace(200, 32, load=1.2, seed=4, median_duration=300)
    cfg = _cfg(nodes=4, gpn=8, gandiva_mem_util=mem)
    s = simulate(cfg, specs, out_dir=str(tmp_path))
    assert s["finished"] + s["failed"] == 200
    assert (tmp_path / "gandiva.csv").exists() and (tmp_path / "job.csv").exists()
    rows = (tmp_path / "gandiva.csv").read_text().splitlines()
    assert rows[0].startswith("time,free_nodes,used_gpus")
