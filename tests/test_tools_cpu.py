"""CLI, profilers, RL environment and utility tests (CPU)."""
import json
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tiresias_amd.config import ClusterSpec, SimConfig
from tiresias_amd.core.job import JobSpec


def test_run_sim_cli_writes_outputs(tmp_path):
    from tiresias_amd.cli import run_sim
    from tiresias_amd.config import FLAGS

    FLAGS.reset()
    s = run_sim.main(["--synthetic", "60", "--schedule", "dlas-gpu", "--scheme", "tiresias",
                      "--num_switch", "1", "--num_node_p_switch", "4", "--num_gpu_p_node", "8",
                      "--queue_limits", "3600", "--log_path", str(tmp_path / "run")])
    assert s["finished"] == 60
    for f in ("cluster.csv", "job.csv", "summary.json", "output.log", "decisions.jsonl"):
        assert (tmp_path / "run" / f).exists()
    FLAGS.reset()


def test_run_sim_reads_reference_trace_schema(tmp_path):
    from tiresias_amd.cli import run_sim
    from tiresias_amd.config import FLAGS
    from tiresias_amd.trace import readers, synth

    p = tmp_path / "tr.csv"
    readers.write_tiresias_trace(str(p), synth.SampleTraceGenerator(0).generate_specs(30, max_gpu=8))
    FLAGS.reset()
    s = run_sim.main(["--trace_file", str(p), "--schedule", "gittins", "--num_node_p_switch", "2",
                      "--log_path", str(tmp_path / "g")])
    assert s["finished"] == 30
    FLAGS.reset()


def test_tick_engine_reference_semantics():
    from tiresias_amd.engine.sim import simulate

    specs = [JobSpec(str(i), float(i), 5.0, 2, gpu_util_avg=10 * i) for i in range(6)]
    c = SimConfig(schedule="horus", scheme="horus", engine="tick",
                  cluster=ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=4))
    s = simulate(c, specs)
    assert s["finished"] == 6
    c2 = SimConfig(schedule="gandiva", scheme="gandiva", engine="tick", timeslice=3,
                   cluster=ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=2))
    s2 = simulate(c2, [JobSpec(str(i), 0.0, 7.0, 2, gpu_mem_max=20000.0) for i in range(3)])
    assert s2["finished"] == 3 and s2["preemptions"] > 0


def test_plot_trace_cdf(tmp_path):
    from tiresias_amd.cli import plot_trace

    rows = plot_trace.main(["--synthetic", "200", "--out", str(tmp_path)])
    assert (tmp_path / "cdf.csv").exists() and rows[0][0] == "duration"


def test_sweep_runs_grid(tmp_path):
    from tiresias_amd.cli import sweep

    res = sweep.main(["--schedules", "fifo,dlas-gpu", "--schemes", "yarn", "--num_queues", "2",
                      "--jobs", "2", "--out", str(tmp_path), "--synthetic", "40",
                      "--num_node_p_switch", "2"])
    assert len(res) == 2 and (tmp_path / "sweep.csv").exists()


def test_scheduling_env_episode():
    from tiresias_amd.engine.env import SchedulingEnv

    specs = [JobSpec(str(i), float(i), 3.0, 1) for i in range(6)]
    env = SchedulingEnv(SimConfig(cluster=ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=2)),
                        specs)
    obs = env.reset()
    total, done, n = 0.0, False, 0
    while not done and n < 1000:
        obs, r, done, info = env.step(0)
        total += r
        n += 1
    assert done and total < 0


def test_memory_estimates_and_utils():
    from tiresias_amd.profiler import memory
    from tiresias_amd.utils import misc

    e = memory.estimate_gpu_memory("vgg16", batch=32)
    assert e["weights_mb"] > 500 and 0 < e["fraction"] < 1
    assert misc.convert_bytes(2 ** 30, "GiB") == 1.0
    assert misc.search_dict_list([{"t": 1}, {"t": 2}], "t", 2) == {"t": 2}
    with pytest.raises(misc.SchedulerError):
        misc.print_fn("boom", misc.LOG_LEVEL_ERROR)


def test_model_profiles_skew():
    from tiresias_amd.profiler.skew import SensitivityOracle, model_profile

    v, r = model_profile("vgg16"), model_profile("resnet50")
    assert v.skew > 0.5 > r.skew                       # VGG's FC layer dominates
    assert 24e6 < r.params < 27e6 and 130e6 < v.params < 145e6
    o = SensitivityOracle(0.5)
    from tiresias_amd.core.job import Job

    assert o(Job(JobSpec("0", 0, 1, 2, model="vgg16"))) and not o(Job(JobSpec("1", 0, 1, 2, model="resnet50")))
    assert model_profile("alexnet").skew > 0.5     # legacy table still served


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _comm_worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tiresias_amd.profiler.comm import CommProfiler

    p = CommProfiler(dist.group.WORLD, device=torch.device("cpu"), iters=2, warmup=1)
    res = p.sweep([0.25, 1.0], {"consolidated": [0, 1], "spread": [0, 2]})
    if rank == 0:
        cls = p.classify_models(["resnet50", "vgg16"], res)
        torch.save({"res": res, "cls": cls}, os.path.join(outdir, "comm.pt"))
    dist.destroy_process_group()


def test_comm_profiler_gloo(tmp_path):
    world = 3
    mp.spawn(_comm_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    d = torch.load(tmp_path / "comm.pt", weights_only=False)
    assert set(d["res"]) == {"consolidated", "spread"} and len(d["res"]["consolidated"]) == 2
    assert d["cls"]["vgg16"]["consolidated_s"] > d["cls"]["resnet50"]["consolidated_s"]


@pytest.mark.parametrize("scenario", ["resnet4", "skew", "seq"])
@pytest.mark.parametrize("n", [1, 2, 8])
def test_bench_scenarios_fit_cluster(scenario, n):
    """bench.py --scenario presets (BASELINE.json configs 2-4): every job fits
    the n-GPU node, ids are unique, arrivals are ordered, and the resnet4
    preset disables LAS demotion (no preemption)."""
    import bench

    jobs = bench.scenario_trace(scenario, n, 2019)
    assert jobs and all(1 <= j.spec.num_gpu <= n for j in jobs)
    assert len({j.spec.job_id for j in jobs}) == len(jobs)
    ts = [j.spec.submit_time for j in jobs]
    assert ts == sorted(ts)
    pol, plc, ck, bpol, bplc, qlim, share = bench.SCENARIOS[scenario]
    cfg = bench.make_cfg(pol, plc, n, 1, ck, qlim, share)
    assert cfg.pack == share
    assert cfg.queue_limits == list(qlim) and cfg.num_queue == len(qlim) + 1
    if scenario == "resnet4":
        assert min(qlim) >= 1e6 and len(jobs) == 4
    if scenario == "seq":
        assert pol == "gittins" and ck == "pressure"


def test_bench_trace_is_scheduler_bound():
    """The headline trace: >= 48 jobs per GPU, offered load above capacity
    (arrival span < nominal work), heavy-tailed, seeded, gangs only when N
    allows, and the Gittins prior comes from a DIFFERENT (held-out) trace."""
    import bench

    for n in (1, 8):
        jobs = bench.bench_trace(n, 48, 2019, work_s=5.0, load=1.6)
        assert len(jobs) == 48 * n and all(1 <= j.spec.num_gpu <= n for j in jobs)
        work = sum(j.spec.duration * j.spec.num_gpu for j in jobs) / n
        span = max(j.spec.submit_time for j in jobs)
        assert 4.5 < work < 5.8 and span < work
        svc = sorted(j.spec.duration for j in jobs)
        assert svc[-1] > 10 * svc[len(svc) // 2]              # heavy tail
        if n == 1:
            assert all(j.spec.num_gpu == 1 for j in jobs)
        else:
            assert any(j.spec.num_gpu > 1 for j in jobs)
    a = bench.bench_trace(1, 48, 2019)
    b = bench.bench_trace(1, 48, 2019)
    assert [(j.model, j.iterations) for j in a] == [(j.model, j.iterations) for j in b]
    h = bench.bench_trace(1, 48, 2019 + bench.HISTORY_SEED_OFFSET)
    assert [j.iterations for j in h] != [j.iterations for j in a]


def test_bench_cpu_driver_contract(tmp_path):
    """``bench.py --cpu --steps 20 --warmup 5`` (the driver's arguments) must
    finish well inside its budget and print one valid JSON line."""
    import json as _json
    import subprocess
    import sys
    import time as _t

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    t = _t.perf_counter()
    # few host threads: under a parallel test run an oversubscribed torch
    # thread pool (not the bench) dominates the wall time
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--cpu", "--steps", "20",
                        "--warmup", "5", "--jobs-per-gpu", "48", "--work-s", "0.05", "--min-iters", "1"],
                       capture_output=True, text=True, timeout=240, cwd=str(tmp_path), env=env)
    wall = _t.perf_counter() - t
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = _json.loads(lines[0])
    assert d["metric"] == bench_metric()
    assert (d["steps"], d["warmup"]) == (20, 5), (d["steps"], d["warmup"], d.get("process_wall_s"))
    assert d["finished_jobs"] == 48 and d["value"] > 0 and d["vs_baseline"] is not None
    assert d["ms_per_step"] * d["steps"] / 1e3 < wall


def bench_metric():
    import bench

    return bench.METRIC


def test_store_grad_arena_layout_and_grad_mode():
    """store_grad params lead the decay region (the optimizer skips zeroing
    [0, n_store)); grad_mode stores the first write of a step and
    accumulates after it; a new optimizer step (grad_epoch) re-arms it."""
    from tiresias_amd.ops import functional as Fx
    from tiresias_amd.ops.arena import Arena

    A = Arena("cpu")
    a = A.add("a", (4, 8))
    s1 = A.add("s1", (16, 8), store_grad=True)
    b = A.add("b", (8,), decay=False, store_grad=True)        # no-decay: never store_grad
    s2 = A.add("s2", (3, 5), store_grad=True)
    A.materialize()
    assert not b.store_grad
    assert [p.name for p in A._order()] == ["s1", "s2", "a", "b"]
    assert s1.offset == 0 and A.n_store == s2.offset + 64 and a.offset == A.n_store
    assert A.n_store <= A.n_decay <= b.offset
    assert Fx.grad_mode(s1) == 0 and Fx.grad_mode(s1) == 1      # first write stores, then accumulate
    assert Fx.grad_mode(a) == 0                                   # (a zeroed param: store == accumulate)
    A.grad_epoch += 1                                             # an optimizer step
    assert Fx.grad_mode(s1) == 0
    old = Fx.STORE_GRAD
    try:
        Fx.STORE_GRAD = False
        A.grad_epoch += 1
        assert Fx.grad_mode(s2) == 1                              # A/B switch: always accumulate
    finally:
        Fx.STORE_GRAD = old
