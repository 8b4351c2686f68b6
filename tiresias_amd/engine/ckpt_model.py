"""Preemption cost model for the simulator (what the real checkpoint engine,
``csrc/ckpt/ckpt_engine.cpp``, costs on MI355X).

Policies:
  none      free and instant (the reference's semantics, ``job.py:49-51``)
  host      every preemption spills the job's state to pinned host DRAM and
            every resume restores it: bytes / ckpt_bw each way
  hbm       the state stays resident in the GPU's HBM while the per-GPU
            suspended-state budget (``ckpt_hbm_budget_gb`` of the 288 GB)
            allows: resume on the same GPUs is free, on other GPUs it is an
            xGMI peer copy; over budget it falls back to the host path
  measured  like ``hbm`` but bandwidths from a measured table
            (``profiles/ckpt_*.json``)
  pressure  the live runtime's policy (``executor/cluster_runtime.Worker``):
            resident until a starting job needs the HBM, then the least
            recently run suspended jobs spill asynchronously; modelled like
            ``hbm`` with the per-GPU budget

Per-GPU state = params x (4 B master + 2 B bf16 shadow + 4/8 B optimizer
state) of the job's model (each DDP replica holds a full copy).
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional, Tuple

from ..profiler.skew import model_profile

XGMI_GBPS = 64.0          # one xGMI link, achievable peer-copy rate


class CkptCostModel:
    def __init__(self, policy: str = "none", host_gbps: float = 50.0, hbm_budget_gb: float = 200.0,
                 table_path: str = ""):
        self.policy = policy
        self.host_gbps = host_gbps
        self.xgmi_gbps = XGMI_GBPS
        self.h2d_gbps = host_gbps
        self.budget = hbm_budget_gb * 1e9
        self.resident: Dict[Tuple[str, int], float] = {}     # (node, dev) -> bytes of suspended state
        self.where: Dict[str, Tuple[str, Optional[dict]]] = {}  # job -> ("hbm"|"host", alloc)
        if table_path and os.path.exists(table_path):
            with open(table_path) as f:
                t = json.load(f)
            self.host_gbps = float(t.get("d2h_gbps") or self.host_gbps)
            self.h2d_gbps = float(t.get("h2d_gbps") or self.host_gbps)
            self.xgmi_gbps = float(t.get("p2p_gbps") or self.xgmi_gbps)

    def state_bytes_per_gpu(self, job) -> float:
        try:
            prof = model_profile(job.spec.model) if job.spec.model else None
        except KeyError:
            prof = None
        if prof is None:
            return 0.0
        opt = "adam" if job.spec.model in ("transformer", "gnmt") else "sgd"
        return float(prof.state_bytes(opt))

    def on_preempt(self, job, alloc) -> Tuple[float, float]:
        """Returns (save seconds, bytes moved)."""
        if self.policy == "none":
            return 0.0, 0.0
        b = self.state_bytes_per_gpu(job)
        total = b * job.num_gpu
        if self.policy in ("hbm", "measured", "pressure") and alloc:
            devs = [(nid, d) for nid, ds in alloc.items() for d in ds]
            if all(self.resident.get(k, 0.0) + b <= self.budget for k in devs):
                for k in devs:
                    self.resident[k] = self.resident.get(k, 0.0) + b
                self.where[job.job_id] = ("hbm", alloc)
                return 0.0, 0.0
        self.where[job.job_id] = ("host", None)
        return b / (self.host_gbps * 1e9), total

    def on_resume(self, job, alloc) -> Tuple[float, float]:
        """Returns (restore seconds, bytes moved)."""
        loc = self.where.pop(job.job_id, None)
        if loc is None or self.policy == "none":
            return 0.0, 0.0
        b = self.state_bytes_per_gpu(job)
        kind, old = loc
        if kind == "hbm":
            for nid, ds in old.items():
                for d in ds:
                    self.resident[(nid, d)] = max(0.0, self.resident.get((nid, d), 0.0) - b)
            if old == alloc:
                return 0.0, 0.0
            return b / (self.xgmi_gbps * 1e9), b * job.num_gpu
        return b / (self.h2d_gbps * 1e9), b * job.num_gpu

    def on_finish(self, job) -> None:
        loc = self.where.pop(job.job_id, None)
        if loc and loc[0] == "hbm":
            b = self.state_bytes_per_gpu(job)
            for nid, ds in loc[1].items():
                for d in ds:
                    self.resident[(nid, d)] = max(0.0, self.resident.get((nid, d), 0.0) - b)
