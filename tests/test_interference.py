"""Measured co-location interference model (replaces the reference's inert
constant FACTOR=0.2, infra/interference.py:1 / node.py:189-204)."""
import json

import pytest

from tiresias_amd.cluster.interference import InterferenceModel
from tiresias_amd.config import ClusterSpec, SimConfig
from tiresias_amd.core.job import JobSpec
from tiresias_amd.engine.sim import simulate


def test_model_pairs_and_fallback(tmp_path):
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"slowdown": {"vgg16|resnet50": 1.9, "resnet50|vgg16": 1.4}}))
    m = InterferenceModel.load(str(p), default_factor=0.2)
    assert m.rate("vgg16", ["resnet50"]) == pytest.approx(1 / 1.9)
    assert m.rate("resnet50", ["vgg16", "gnmt"]) == pytest.approx(1 / 1.4)   # worst neighbour (1.4 > 1.2)
    assert m.rate("gnmt", ["bert"]) == pytest.approx(1 / 1.2)                  # constant fallback
    assert m.rate("vgg_tiny", ["resnet_tiny"]) == pytest.approx(1 / 1.9)       # tiny variants map to base
    assert m.rate("vgg16", []) == 1.0


def test_simulator_uses_measured_pairs(tmp_path):
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"slowdown": {"vgg16|resnet50": 2.0, "resnet50|vgg16": 1.25}}))
    spec = ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=1, gpu_memory_mb=288 * 1024)
    jobs = [JobSpec("a", 0.0, 100.0, 1, model="vgg16", gpu_mem_max=1000),
            JobSpec("b", 0.0, 100.0, 1, model="resnet50", gpu_mem_max=1000)]
    cfg = SimConfig(schedule="fifo", scheme="pack", pack=True, interference_table=str(p), cluster=spec)
    s = simulate(cfg, jobs)
    assert s["finished"] == 2
    # b runs at 1/1.25 while sharing; a at 1/2: b ends first at 125 s (a has done 62.5),
    # then a runs alone for 37.5 s more -> 162.5 s
    assert s["makespan"] == pytest.approx(162.5, rel=1e-6)


def test_measured_spread_slowdown_drives_progress_rate(tmp_path):
    """With --enable_network_costs and a measured skew profile, a gang spread
    over two (virtual) nodes progresses at 1/slowdown measured for its model
    (profiler/comm.py output), not the analytic ring formula; a model the
    profile does not cover keeps the analytic rate."""
    import json

    from tiresias_amd.cluster.network import measured_spread_rate
    from tiresias_amd.config import ClusterSpec, SimConfig
    from tiresias_amd.core.job import JobSpec
    from tiresias_amd.engine.sim import Simulator

    assert measured_spread_rate(1.5, 1) == 1.0
    assert abs(measured_spread_rate(1.5, 2) - 1 / 1.5) < 1e-12
    assert measured_spread_rate(1.5, 4) < measured_spread_rate(1.5, 2)      # ring: 2(k-1)/k
    path = tmp_path / "skew.json"
    path.write_text(json.dumps({"vgg16": {"slowdown": 1.6, "sensitive": True}}))
    cfg = SimConfig(schedule="fifo", scheme="yarn", skew_profile=str(path), enable_network_costs=True,
                    cluster=ClusterSpec(num_switch=1, num_node_p_switch=2, num_gpu_p_node=4))
    # 6 GPUs cannot fit one 4-GPU node: yarn spreads the gang over both nodes
    sim = Simulator(cfg, [JobSpec("v", 0.0, 16.0, 6, model="vgg16")])
    s = sim.run()
    assert abs(sim.jobs["v"].end_time - 16.0 * 1.6) < 1e-6, s
