"""Typed configuration for the scheduler, simulator and cluster runtime.

Flag names keep the reference CLI (``/root/reference/run_sim.py:19-93``):
trace_file, log_path, scheme, schedule, pack, num_switch, num_node_p_switch,
enable_network_costs, enable_migration, bandwidth, internode_latency,
gpu_memory_capacity, num_queue, num_gpu_p_node, num_cpu_p_node, mem_p_node,
cluster_spec, print, flush_stdout. New ones cover what the reference hard-coded
or lacked (queue_limits, solve_starvation, gittins_delta, gittins_prior, seed,
backend, ckpt model, virtual nodes, time unit, ...).
"""
from __future__ import annotations

import csv
import os
from dataclasses import asdict, dataclass, field, fields
from typing import List, Optional

from . import flags as _fl
from .flags import FLAGS


def define_flags() -> None:
    if "schedule" in FLAGS:
        return
    D = _fl
    # ---- reference flags (run_sim.py:19-93) ----
    D.DEFINE_string("trace_file", "", "job trace (*.csv); schema auto-detected (philly / tiresias)")
    D.DEFINE_string("log_path", "", "output folder (default log/result-<timestamp>)")
    D.DEFINE_string("scheme", "yarn", "placement: count|yarn|random|crandom|greedy|balance|cbalance|"
                    "horus|horus+|gandiva|pack|tiresias|lp")
    D.DEFINE_string("schedule", "fifo", "policy: fifo|fjf|sjf|lpjf|shortest|shortest-gpu|"
                    "shortest-expected|dlas|dlas-gpu|dlas-gpu-gittins|gittins|multi-dlas-gpu|"
                    "dlas-gpu-pack|horus|horus+|gandiva|gandiva-ns (legacy node-set engine)")
    D.DEFINE_boolean("pack", False, "allow GPU sharing (co-location) in placement")
    D.DEFINE_integer("num_switch", 1, "racks (switches)")
    D.DEFINE_integer("num_node_p_switch", 32, "nodes per rack")
    D.DEFINE_boolean("enable_network_costs", False, "slow spread jobs by the comm model")
    D.DEFINE_boolean("enable_migration", False, "migrate tasks off overloaded devices")
    D.DEFINE_integer("bandwidth", 1250, "inter-node bandwidth per rack, MB/s")
    D.DEFINE_float("internode_latency", 0.015, "inter-node latency, seconds")
    D.DEFINE_integer("gpu_memory_capacity", 32, "GPU memory, GiB")
    D.DEFINE_integer("num_queue", 1, "number of priority queues (MLFQ / horus+ clusters)")
    D.DEFINE_integer("num_gpu_p_node", 8, "GPUs per node")
    D.DEFINE_integer("num_cpu_p_node", 128, "CPU cores per node")
    D.DEFINE_integer("mem_p_node", 512, "host memory per node, GiB")
    D.DEFINE_string("cluster_spec", "", "cluster spec csv (overrides the topology flags)")
    D.DEFINE_boolean("print", False, "verbose decision log to stdout")
    D.DEFINE_boolean("flush_stdout", True, "flush stdout")
    # ---- new ----
    D.DEFINE_list("queue_limits", [], "MLFQ demotion thresholds (service units), e.g. 3600,7200")
    D.DEFINE_float("solve_starvation", 0.0, "promote to Q0 when pending >= executed * this (0=off)")
    D.DEFINE_float("gittins_delta", 3250.0, "Gittins quantum (service units)")
    D.DEFINE_string("gittins_prior", "", "history csv with a duration column (GPU-service) for the "
                    "Gittins / expected-remaining prior (reference yarn-gput1000.csv)")
    D.DEFINE_string("prior_mode", "online", "without --gittins_prior: online (learn from finished jobs) | "
                    "oracle (the replayed trace's own distribution; flagged in summary.json)")
    D.DEFINE_integer("seed", 0, "RNG seed (all randomness is seeded)")
    D.DEFINE_string("backend", "sim", "sim: discrete-event simulator | fake: the live controller against "
                    "a virtual-time executor (executor/fake.py) | mi355x: live GPUs (cli/run_cluster)")
    D.DEFINE_string("engine", "event", "event (discrete-event) | tick (reference-compatible tick loop)")
    D.DEFINE_float("time_unit", 1.0, "seconds per trace time unit")
    D.DEFINE_float("duration_scale", 1.0, "scale applied to trace durations")
    D.DEFINE_string("ckpt_policy", "none", "none | hbm | host | measured | pressure: preemption state "
                    "(pressure: resident in HBM, spilled to pinned host only when a starting job needs the HBM)")
    D.DEFINE_float("ckpt_bw_gbps", 50.0, "spill/restore bandwidth GB/s for ckpt_policy=host")
    D.DEFINE_float("ckpt_hbm_budget_gb", 200.0, "HBM per GPU reserved for suspended jobs")
    D.DEFINE_string("ckpt_table", "profiles/ckpt_mi355x.json",
                    "measured spill/restore/peer bandwidths for ckpt_policy=measured (python -m tiresias_amd.ckpt)")
    D.DEFINE_string("virtual_nodes", "", "partition the MI355X box, e.g. 2x4 or 4x2")
    D.DEFINE_float("nic_gbps", 12.5, "inter-virtual-node link rate per GPU, GB/s (spread gangs' "
                   "host-staged transport, parallel/gang.py)")
    D.DEFINE_string("skew_profile", "", "JSON of measured consolidated-vs-spread all-reduce slowdowns "
                    "per model (python -m tiresias_amd.profiler.comm); drives placement sensitivity")
    D.DEFINE_float("interference", 0.2, "co-location slowdown factor (reference infra/interference.py)")
    D.DEFINE_string("interference_table", "", "measured per-model-pair slowdowns (JSON from "
                    "tools/measure_interference.py); overrides the constant factor per pair")
    D.DEFINE_integer("max_tasks_per_gpu", 3, "co-location limit per GPU")
    D.DEFINE_boolean("gang_align", False, "place power-of-two gangs on aligned buddy device blocks "
                     "(canonical rank sets: bounded, pre-created RCCL communicators; live runtime)")
    D.DEFINE_float("gpu_mem_headroom_mb", 500.0, "free memory a GPU must keep when packing")
    D.DEFINE_integer("lookahead", 5, "horus/horus+ look-ahead window")
    D.DEFINE_float("timeslice", 100.0, "gandiva time-slice quantum (time units)")
    D.DEFINE_float("replan_interval", 600.0, "multi-dlas reservation re-plan interval")
    D.DEFINE_float("gandiva_tick", 10.0, "gandiva-ns: engine tick (s)")
    D.DEFINE_float("gandiva_slice", 60.0, "gandiva-ns: time-slice rotation period (s)")
    D.DEFINE_string("gandiva_mem_util", "one", "gandiva-ns job slot size: one|legacy|measured")
    D.DEFINE_boolean("replace_all", False, "re-place every runnable job at each event (legacy Tiresias)")
    D.DEFINE_float("skew_threshold", 0.5, "placement-sensitivity threshold (largest tensor / total)")
    D.DEFINE_string("spread_rule", "node", "tiresias placement, insensitive gangs: fragments (spread "
                    "whenever no consolidated block is free) | wait (spread only when the expected wait "
                    "for a block exceeds the spread penalty, engine/spread.py) | price (as wait, the penalty "
                    "also charging the queued gangs the fragments delay) | node (as wait, but a gang "
                    "that fits one node is never fragmented and a wider gang fills the fullest-free "
                    "nodes first)")
    D.DEFINE_string("preempt_rule", "lazy", "preemptive policies: lazy (preempt only what a chosen job's "
                    "placement needs) | eager (every running job outside the priority prefix)")
    D.DEFINE_boolean("ddp_shard", False, "live gangs: reduce-scatter + sharded optimizer + bf16 all-gather "
                     "(consolidated on suspension)")
    D.DEFINE_string("ddp_wire", "fp32", "sharded gangs: reduce-scatter wire dtype fp32 | bf16")
    D.DEFINE_string("throughput_table", "", "json of measured per-model iteration times (MI355X)")
    D.DEFINE_integer("max_jobs", 0, "truncate the trace (0 = all)")
    D.DEFINE_integer("debug_kernels", 0, "kernel debug mode (utils/debug.py): 1 synchronous launches "
                     "+ per-op HIP error check, 2 also NaN/Inf checks of every op's outputs")
    D.DEFINE_version("0.1.0")


@dataclass
class ClusterSpec:
    num_switch: int = 1
    num_node_p_switch: int = 32
    num_gpu_p_node: int = 8
    num_cpu_p_node: int = 128
    mem_p_node: int = 512
    gpu_memory_mb: float = 32 * 1024
    bandwidth_mbps: float = 1250.0
    internode_latency: float = 0.015

    @property
    def num_nodes(self) -> int:
        return self.num_switch * self.num_node_p_switch

    @property
    def num_gpus(self) -> int:
        return self.num_nodes * self.num_gpu_p_node

    @staticmethod
    def from_csv(path: str, base: Optional["ClusterSpec"] = None) -> "ClusterSpec":
        """Reference format ``cluster_spec.csv:1-2`` (header + one row)."""
        spec = base or ClusterSpec()
        with open(path) as f:
            rows = list(csv.DictReader(f))
        if len(rows) != 1:
            raise ValueError(f"{path}: expected exactly one spec row, got {len(rows)}")
        r = rows[0]
        for k in ("num_switch", "num_node_p_switch", "num_gpu_p_node", "num_cpu_p_node", "mem_p_node"):
            if k in r and r[k] != "":
                v = int(r[k])
                if v <= 0:
                    raise ValueError(f"{path}: {k} must be positive")
                setattr(spec, k, v)
        return spec

    @staticmethod
    def mi355x_node() -> "ClusterSpec":
        """One 8x MI355X node: 288 GB HBM3E per GPU, fully connected xGMI."""
        return ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=8, num_cpu_p_node=128,
                           mem_p_node=3072, gpu_memory_mb=288 * 1024, bandwidth_mbps=153_000.0,
                           internode_latency=5e-6)


@dataclass
class SimConfig:
    schedule: str = "fifo"
    scheme: str = "yarn"
    pack: bool = False
    num_queue: int = 1
    queue_limits: List[float] = field(default_factory=list)
    solve_starvation: float = 0.0
    gittins_delta: float = 3250.0
    gittins_prior: str = ""
    prior_mode: str = "online"        # no prior file: online (finished jobs) | oracle (trace itself)
    seed: int = 0
    engine: str = "event"
    time_unit: float = 1.0
    duration_scale: float = 1.0
    ckpt_policy: str = "none"
    ckpt_bw_gbps: float = 50.0
    ckpt_hbm_budget_gb: float = 200.0
    ckpt_table: str = "profiles/ckpt_mi355x.json"
    enable_network_costs: bool = False
    enable_migration: bool = False
    interference: float = 0.2
    interference_table: str = ""
    max_tasks_per_gpu: int = 3
    gang_align: bool = False          # canonical (buddy-aligned) gang rank sets
    gpu_mem_headroom_mb: float = 500.0
    lookahead: int = 5
    timeslice: float = 100.0
    replan_interval: float = 600.0
    gandiva_tick: float = 10.0
    gandiva_slice: float = 60.0
    gandiva_mem_util: str = "one"
    replace_all: bool = False
    skew_threshold: float = 0.5
    spread_rule: str = "node"          # tiresias placement: node | wait | price | fragments (engine/spread.py)
    preempt_rule: str = "lazy"         # preemptive policies: lazy | eager (engine/sim.py::_schedule_lazy)
    ddp_shard: bool = False            # live gangs: sharded data parallelism (parallel/ddp.py)
    ddp_wire: str = "fp32"             # sharded gangs: reduce-scatter dtype fp32 | bf16
    virtual_nodes: str = ""
    nic_gbps: float = 12.5            # emulated inter-virtual-node link per GPU (GB/s)
    skew_profile: str = ""            # measured consolidated-vs-spread slowdowns (profiler/comm.py)
    throughput_table: str = ""
    log_path: str = ""
    verbose: bool = False
    cluster: ClusterSpec = field(default_factory=ClusterSpec)

    @staticmethod
    def from_flags(fl=FLAGS) -> "SimConfig":
        define_flags()
        d = fl.as_dict()
        spec = ClusterSpec(num_switch=d["num_switch"], num_node_p_switch=d["num_node_p_switch"],
                           num_gpu_p_node=d["num_gpu_p_node"], num_cpu_p_node=d["num_cpu_p_node"],
                           mem_p_node=d["mem_p_node"], gpu_memory_mb=d["gpu_memory_capacity"] * 1024.0,
                           bandwidth_mbps=float(d["bandwidth"]), internode_latency=d["internode_latency"])
        if d.get("cluster_spec") and os.path.exists(d["cluster_spec"]):
            spec = ClusterSpec.from_csv(d["cluster_spec"], spec)
        names = {f.name for f in fields(SimConfig)}
        kw = {k: v for k, v in d.items() if k in names and k != "cluster"}
        kw["queue_limits"] = [float(x) for x in d.get("queue_limits") or []]
        kw["verbose"] = bool(d.get("print"))
        return SimConfig(cluster=spec, **kw)

    def to_dict(self):
        return asdict(self)
