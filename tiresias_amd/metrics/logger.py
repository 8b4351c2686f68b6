"""Simulation / cluster-run outputs.

Keeps both reference CSV schemas (``/root/reference/log_manager.py:36-43,
105-108``) and actually WRITES them (defect D5: the live reference creates
header-only job/cpu/gpu/memory/network CSVs):

* ``cluster.csv`` — one row per scheduling event: delta, idle/busy nodes,
  busy/idle GPUs, avg GPU utilisation (a float in [0,100], defect D9), avg GPU
  memory allocated, avg/median/max pending time, running/queuing/finished;
* ``job.csv`` — one row per finished job with JCT (legacy ``log.py:316-330``
  columns + migration, queue, checkpoint overhead/bytes, model);
* ``gpu.csv`` / ``cpu.csv`` / ``memory.csv`` / ``network.csv`` — per-node
  utilisation snapshots each event;
* ``decisions.jsonl`` — one record per scheduler decision;
* ``summary.json`` — avg / median / p95 JCT, makespan, queueing delay, GPU
  utilisation (time-weighted), preemptions, migrations, checkpoint bytes.
"""
from __future__ import annotations

import csv
import json
import os
import statistics
from typing import Dict, List, Optional

CLUSTER_HEADER = ["delta", "num_idle_nodes", "num_busy_nodes", "num_busy_gpus", "num_idle_gpus",
                  "avg_gpu_utilization", "avg_gpu_memory_allocated", "avg_pending_time",
                  "median_pending_time", "max_pending_time", "num_running_jobs", "num_queuing_jobs",
                  "num_finish_jobs"]
JOB_HEADER = ["time", "job_id", "num_gpu", "submit_time", "start_time", "end_time", "executed_time",
              "JCT", "duration", "pending_time", "preempt", "resume", "promote", "migration",
              "queue", "ckpt_overhead", "ckpt_bytes", "ckpt_save_s", "ckpt_restore_s", "comm_exposed_s",
              "comm_span_s", "comm_bytes_per_step", "gather_exposed_s", "gather_window_s", "model", "lost_iters"]


def percentile(xs: List[float], p: float) -> float:
    if not xs:
        return 0.0
    s = sorted(xs)
    k = (len(s) - 1) * p / 100.0
    lo = int(k)
    hi = min(lo + 1, len(s) - 1)
    return s[lo] + (s[hi] - s[lo]) * (k - lo)


class MetricsLogger:
    def __init__(self, out_dir: Optional[str] = None, node_logs: bool = True, decisions: bool = True):
        self.out_dir = out_dir
        self.node_logs = node_logs and out_dir is not None
        self.cluster_rows: List[list] = []
        self.job_rows: List[dict] = []
        self._files = {}
        self._writers = {}
        self._dec = None
        if out_dir:
            os.makedirs(out_dir, exist_ok=True)
            self._open("cluster", CLUSTER_HEADER)
            self._open("job", JOB_HEADER)
            if self.node_logs:
                self._open("gpu", ["delta", "node", "device", "num_tasks", "utilization", "memory_used"])
                self._open("cpu", ["delta", "node", "cpu_used", "cpu_count"])
                self._open("memory", ["delta", "node", "mem_used", "mem_size"])
                self._open("network", ["delta", "job_id", "num_nodes", "rate"])
            if decisions:
                # line-buffered: a post-mortem of a wedged / killed run keeps every decision
                self._dec = open(os.path.join(out_dir, "decisions.jsonl"), "w", buffering=1)
        self.busy_gpu_time = 0.0
        self.last_t = None
        self.last_busy = 0
        self.counters = dict(preempt=0, migrate=0, start=0, finish=0, failed=0)

    def _open(self, name, header):
        f = open(os.path.join(self.out_dir, f"{name}.csv"), "w", newline="")
        w = csv.writer(f)
        w.writerow(header)
        self._files[name] = f
        self._writers[name] = w

    # ------------------------------------------------------------------ events
    def decision(self, t: float, ev: str, job_id: str, **kw) -> None:
        if ev in self.counters:
            self.counters[ev] += 1
        if self._dec:
            rec = {"t": round(t, 6), "ev": ev, "job": job_id}
            rec.update(kw)
            self._dec.write(json.dumps(rec) + "\n")

    def account(self, t: float, busy_gpus: int) -> None:
        if self.last_t is not None and t > self.last_t:
            self.busy_gpu_time += self.last_busy * (t - self.last_t)
        self.last_t = t
        self.last_busy = busy_gpus

    def cluster_row(self, t: float, cluster, jobs_pending, n_running: int, n_finished: int) -> None:
        idle_nodes = sum(1 for n in cluster.nodes.values() if n.is_idle())
        busy_nodes = len(cluster.nodes) - idle_nodes
        busy_g = cluster.busy_gpus()
        idle_g = cluster.num_gpus - busy_g
        utils, mem_used, mem_cap = [], 0.0, 0.0
        for n in cluster.nodes.values():
            for d in n.devices:
                utils.append(d.utilization() if d.tasks else 0.0)
                mem_used += d.memory_used()
                mem_cap += d.memory
        pend = [j.pending_time for j in jobs_pending]
        row = [round(t, 6), idle_nodes, busy_nodes, busy_g, idle_g,
               round(sum(utils) / max(1, len(utils)), 4), round(mem_used / max(1.0, mem_cap), 6),
               round(sum(pend) / len(pend), 4) if pend else 0.0,
               round(statistics.median(pend), 4) if pend else 0.0,
               round(max(pend), 4) if pend else 0.0, n_running, len(pend), n_finished]
        self.cluster_rows.append(row)
        if "cluster" in self._writers:
            self._writers["cluster"].writerow(row)
        if self.node_logs:
            for n in cluster.nodes.values():
                for d in n.devices:
                    self._writers["gpu"].writerow([round(t, 6), n.node_id, d.device_id, len(d.tasks),
                                                   round(d.utilization(), 3), round(d.memory_used(), 1)])
                self._writers["cpu"].writerow([round(t, 6), n.node_id, n.cpu_used, n.cpu_count])
                self._writers["memory"].writerow([round(t, 6), n.node_id, n.mem_used, n.mem_size])

    def device_row(self, t: float, rank: int, util_pct, free_mb, total_mb, job_id) -> None:
        """Live runtime: measured state of one rank's GPU (hipMemGetInfo +
        amd-smi activity), replacing the reference's sampled utilisation."""
        if not self.out_dir:
            return
        if "gpu_live" not in self._writers:
            self._open("gpu_live", ["time", "rank", "util_pct", "free_mb", "total_mb", "job_id"])
        self._writers["gpu_live"].writerow([round(t, 6), rank, "" if util_pct is None else util_pct,
                                            free_mb, total_mb, job_id or ""])

    GANDIVA_CLASSES = (1, 2, 4, 8, 16, 32, 64)

    def gandiva_row(self, t: float, free_nodes: int, used_gpus: int, idle_gpus: int, n_pending: int,
                    n_running: int, sets_per_class: Dict[int, int]) -> None:
        """Node-set engine row (reference ``log.py`` gandiva checkpoint):
        free nodes, used / idle GPUs, pending / running jobs, #sets per class."""
        if not self.out_dir:
            return
        if "gandiva" not in self._writers:
            self._open("gandiva", ["time", "free_nodes", "used_gpus", "idle_gpus", "pending_jobs",
                                   "running_jobs"] + [f"node_g{g}" for g in self.GANDIVA_CLASSES])
        self._writers["gandiva"].writerow([round(t, 6), free_nodes, used_gpus, idle_gpus, n_pending,
                                           n_running] + [sets_per_class.get(g, 0)
                                                         for g in self.GANDIVA_CLASSES])

    def network_row(self, t: float, job_id: str, nodes: int, rate: float) -> None:
        if self.node_logs:
            self._writers["network"].writerow([round(t, 6), job_id, nodes, round(rate, 6)])

    def job_row(self, t: float, j) -> None:
        row = dict(time=round(t, 6), job_id=j.job_id, num_gpu=j.num_gpu,
                   submit_time=round(j.spec.submit_time, 6),
                   start_time=round(j.start_time, 6) if j.start_time is not None else "",
                   end_time=round(j.end_time, 6) if j.end_time is not None else "",
                   executed_time=round(j.total_executed, 6),
                   JCT=round(j.jct, 6) if j.jct is not None else "",
                   duration=round(j.spec.duration, 6), pending_time=round(j.pending_time, 6),
                   preempt=j.preempt_count, resume=j.resume_count, promote=j.promote_count,
                   migration=j.migration_count, queue=j.queue,
                   ckpt_overhead=round(j.overhead_time, 6), ckpt_bytes=int(j.ckpt_bytes),
                   # measured on the live cluster (device copy time of spills / restores)
                   ckpt_save_s=round(j.extra.get("ckpt_save_s", 0.0), 6),
                   # iterations redone after a failure (restart from the last
                   # snapshot, or from scratch without one)
                   lost_iters=int(j.extra.get("lost_iters", 0)),
                   ckpt_restore_s=round(j.extra.get("ckpt_restore_s", 0.0), 6),
                   comm_exposed_s=round(j.extra.get("comm_exposed_s", 0.0), 6),
                   comm_span_s=round(j.extra.get("comm_span_s", 0.0), 6),
                   comm_bytes_per_step=(int(j.extra["comm_bytes"] / j.extra["comm_steps"])
                                        if j.extra.get("comm_steps") else 0),
                   gather_exposed_s=round(j.extra.get("gather_exposed_s", 0.0), 6),
                   gather_window_s=round(j.extra.get("gather_window_s", 0.0), 6),
                   model=j.spec.model)
        self.job_rows.append(row)
        if "job" in self._writers:
            self._writers["job"].writerow([row[k] for k in JOB_HEADER])

    # ------------------------------------------------------------------ summary
    def summary(self, jobs, num_gpus: int, wall_s: float = 0.0, extra: Optional[Dict] = None) -> Dict:
        done = [j for j in jobs if j.end_time is not None]
        jcts = [j.jct for j in done]
        waits = [(j.start_time - j.spec.submit_time) for j in done if j.start_time is not None]
        t0 = min((j.spec.submit_time for j in jobs), default=0.0)
        makespan = (max((j.end_time for j in done), default=0.0) - t0) if done else 0.0
        s = dict(
            jobs=len(jobs), finished=len(done), failed=sum(1 for j in jobs if j.state.name == "FAILED"),
            avg_jct=statistics.fmean(jcts) if jcts else 0.0,
            median_jct=statistics.median(jcts) if jcts else 0.0,
            p95_jct=percentile(jcts, 95), max_jct=max(jcts) if jcts else 0.0,
            makespan=makespan,
            avg_queueing_delay=statistics.fmean(waits) if waits else 0.0,
            avg_pending_time=statistics.fmean([j.pending_time for j in done]) if done else 0.0,
            gpu_utilization=(self.busy_gpu_time / (num_gpus * makespan)) if makespan > 0 else 0.0,
            preemptions=sum(j.preempt_count for j in jobs),
            migrations=sum(j.migration_count for j in jobs),
            promotions=sum(j.promote_count for j in jobs),
            ckpt_bytes=float(sum(j.ckpt_bytes for j in jobs)),
            ckpt_overhead_s=float(sum(j.overhead_time for j in jobs)),
            wall_s=wall_s,
        )
        if extra:
            s.update(extra)
        if self.out_dir:
            with open(os.path.join(self.out_dir, "summary.json"), "w") as f:
                json.dump(s, f, indent=1, sort_keys=True)
        return s

    def close(self) -> None:
        for f in self._files.values():
            f.close()
        self._files = {}
        self._writers = {}
        if self._dec:
            self._dec.close()
            self._dec = None
