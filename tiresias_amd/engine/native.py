"""Python front-end of the native event core (``csrc/sched_core``).

``simulate_native(cfg, specs)`` returns the same summary dict as
``engine.sim.simulate`` for the policies the core implements under the
``count`` (flat GPU pool), ``yarn`` (consolidated, per-node CPU / memory,
rack-aware cross-node) and ``tiresias`` (skew-aware: sensitive models
consolidated, insensitive ones on fragments) placements -- the reference's
sweep configuration (``execute.py:44-53``: 4 switches x 32 nodes, a month
trace) -- and is cross-checked job-for-job against the Python engine
(tests/test_sched_core.py). Use it for month-scale trace sweeps.
"""
from __future__ import annotations

import statistics
import time
from typing import Dict, List, Optional

import numpy as np

from ..config import SimConfig
from ..core.job import JobSpec
from ..metrics.logger import percentile

SUPPORTED = ("fifo", "fjf", "sjf", "shortest", "shortest-gpu", "dlas", "dlas-gpu", "dlas-gpu-gittins",
             "gittins")
PLACEMENTS = ("count", "yarn", "tiresias")


def available() -> bool:
    try:
        from .. import _sched_core  # noqa: F401
        return True
    except ImportError:
        return False


def simulate_native(cfg: SimConfig, specs: List[JobSpec], prior: Optional[List[float]] = None) -> Dict:
    from .. import _sched_core
    from ..policy.las import default_limits

    if cfg.schedule not in SUPPORTED:
        raise ValueError(f"native core supports {SUPPORTED}, not {cfg.schedule}")
    scheme = cfg.scheme if cfg.scheme not in ("", "default") else "count"
    if scheme not in PLACEMENTS:
        raise ValueError(f"native core placements are {PLACEMENTS}, not {scheme}")
    if cfg.pack or cfg.virtual_nodes or getattr(cfg, "gang_align", False) or cfg.enable_migration:
        raise ValueError("native core: no GPU sharing, virtual nodes or gang alignment (use engine.sim)")
    limits = list(cfg.queue_limits) or default_limits(cfg.num_queue if cfg.num_queue > 1 else 2, 3600.0)
    # prior: same rules as engine/sim.py::Simulator._prior (history, never the future)
    source = "explicit"
    if prior is None and cfg.gittins_prior:
        from ..trace.readers import read_duration_prior

        prior, source = read_duration_prior(cfg.gittins_prior), "file"
    elif prior is None and cfg.prior_mode == "oracle":
        prior, source = sorted(s.duration * s.num_gpu for s in specs), "oracle"
    online = prior is None
    if online:
        prior, source = [], "online"
    eng = _sched_core.Engine(cfg.schedule, cfg.cluster.num_gpus, [float(x) for x in limits],
                             float(cfg.solve_starvation), float(cfg.gittins_delta or 3250.0),
                             [float(x) for x in prior], online)
    rule = getattr(cfg, "spread_rule", "node")
    if rule not in ("node", "wait", "fragments", "price"):
        raise ValueError(f"spread_rule must be node | wait | price | fragments, got {rule!r}")
    wait_rule = scheme == "tiresias" and rule in ("wait", "node", "price")
    priced = _set_costs(eng, cfg, specs, force=wait_rule)
    eng.set_spread_wait(wait_rule)
    eng.set_spread_node(scheme == "tiresias" and rule == "node")
    eng.set_spread_price(scheme == "tiresias" and rule == "price")
    eng.set_lazy_preempt(getattr(cfg, "preempt_rule", "lazy") == "lazy")
    t0 = time.perf_counter()
    sub_a = np.array([s.submit_time for s in specs], dtype=np.float64)
    dur_a = np.array([s.duration for s in specs], dtype=np.float64)
    gpu_a = np.array([s.num_gpu for s in specs], dtype=np.int32)
    if scheme == "count" and not priced:
        out = eng.run(sub_a, dur_a, gpu_a)
    else:
        c = cfg.cluster
        eng.set_topology(scheme, c.num_switch, c.num_node_p_switch, c.num_gpu_p_node, c.num_cpu_p_node,
                         c.mem_p_node)
        sens = np.zeros(len(specs), dtype=np.uint8)
        if scheme == "tiresias":
            # the same oracle the Python engine consults (measured skew
            # profile if configured, else the model's largest-tensor ratio)
            from ..core.job import Job
            from ..profiler.skew import SensitivityOracle

            oracle = SensitivityOracle(cfg.skew_threshold, measured_path=cfg.skew_profile)
            sens = np.array([1 if oracle(Job(s)) else 0 for s in specs], dtype=np.uint8)
        out = eng.run_topo(sub_a, dur_a, gpu_a,
                           np.array([s.gpu_per_worker for s in specs], dtype=np.int32),
                           np.array([s.cpu_per_task for s in specs], dtype=np.int32),
                           np.array([s.mem_per_task for s in specs], dtype=np.int32), sens)
    wall = time.perf_counter() - t0
    cost = eng.costs() if priced else None
    sub = np.array([s.submit_time for s in specs])
    end, start = out["end"], out["start"]
    done = end >= 0
    jct = (end - sub)[done]
    t_first = float(sub.min()) if len(sub) else 0.0
    return dict(jobs=len(specs), finished=int(done.sum()), failed=int((~done).sum()),
                avg_jct=float(jct.mean()) if len(jct) else 0.0,
                median_jct=float(statistics.median(jct.tolist())) if len(jct) else 0.0,
                p95_jct=percentile(jct.tolist(), 95), makespan=float(end.max() - t_first) if done.any() else 0.0,
                avg_queueing_delay=float((start - sub)[done].mean()) if done.any() else 0.0,
                preemptions=int(out["preempt"].sum()), promotions=int(out["promote"].sum()),
                events=int(out["events"]), wall_s=wall, schedule=cfg.schedule, scheme=scheme, prior=source,
                priced=priced,
                ckpt_overhead_s=float(cost["overhead"].sum()) if cost is not None else 0.0,
                ckpt_gb=float(cost["ckpt_bytes"].sum() / 1e9) if cost is not None else 0.0,
                per_job={"start": start, "end": end, "preempt": out["preempt"],
                         **({"overhead": cost["overhead"], "ckpt_bytes": cost["ckpt_bytes"]}
                            if cost is not None else {})})


CKPT_MODE = {"none": 0, "host": 1, "hbm": 2, "measured": 2, "pressure": 2}


def _set_costs(eng, cfg: SimConfig, specs: List[JobSpec], force: bool = False) -> bool:
    """Price the replay like the Python engine: the per-job parameters of
    engine/sim.py::Simulator._rate (measured 2-node slowdown, else the
    analytic all-reduce over the link) and engine/ckpt_model.py (state bytes
    per GPU, bandwidths -- the measured table for ckpt_policy=measured).
    ``force``: hand over the per-job spread parameters even when nothing is
    charged (the wait-vs-spread placement rule estimates with them).
    Returns whether any cost is on."""
    net = bool(cfg.enable_network_costs)
    mode = CKPT_MODE.get(cfg.ckpt_policy)
    if mode is None:
        raise ValueError(f"native core: unsupported ckpt_policy {cfg.ckpt_policy}")
    if not net and mode == 0 and not force:
        return False
    from ..core.job import Job
    from ..profiler.skew import SensitivityOracle, model_profile
    from .ckpt_model import CkptCostModel

    ck = CkptCostModel(cfg.ckpt_policy, cfg.ckpt_bw_gbps, cfg.ckpt_hbm_budget_gb,
                       table_path=cfg.ckpt_table if cfg.ckpt_policy == "measured" else "")
    oracle = SensitivityOracle(cfg.skew_threshold, measured_path=cfg.skew_profile)
    ckpt_b, sd, it_s, nbytes = [], [], [], []
    for s in specs:
        j = Job(s)
        ckpt_b.append(float(ck.state_bytes_per_gpu(j)))
        m = s.model or ""
        v = oracle.slowdown(m)
        sd.append(float(v) if v is not None else -1.0)
        # cluster/network.py::network_rate's inputs
        try:
            mb = model_profile(m).total_mb if m else 100.0
        except KeyError:
            mb = 100.0
        it_s.append(s.duration / s.iterations if s.iterations and s.iterations > 0 else 0.25)
        nbytes.append(mb * 2 ** 20)
    c = cfg.cluster
    eng.set_costs(net, float(c.bandwidth_mbps), float(c.internode_latency), mode, float(ck.host_gbps),
                  float(ck.h2d_gbps), float(ck.xgmi_gbps), float(ck.budget), ckpt_b, sd, it_s, nbytes)
    return net or mode != 0
