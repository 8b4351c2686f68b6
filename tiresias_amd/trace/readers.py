"""Trace ingest: both reference schemas plus the Gittins prior.

* Philly / NSDI'19 "live" schema (reference ``core/jobs/job_generator.py:
  165-207`` + ``jobs_manager.py:225-238``): ``type, normalized_time, minutes,
  gpu_per_container, used_gpus, gpu_utilization_avg, gpu_utilization_max,
  memory_avg, memory_max`` (memory in bytes). Rows with type != noninteractive
  are dropped, NaN rows dropped, time rebased to 0 and divided by
  ``time_div`` (reference: 10000); duration = minutes * ``minutes_scale``
  (reference tick loop: 0.5).
* Tiresias schema (reference ``README.md:17-25``): ``job_id, num_gpu,
  submit_time, iterations, model_name, duration, interval`` (seconds).
* Gittins / expected-remaining prior: any csv with a ``duration`` column
  (reference ``run_sim.py:1682-1707``).

Readers return sorted ``JobSpec`` lists; ``StreamingReader`` releases rows by
time with an index cursor (O(new rows) per call, not the reference's O(N)
pandas mask per tick).
"""
from __future__ import annotations

import csv
import math
import os
from typing import Iterable, List, Optional

from ..core.job import JobSpec

LIVE_COLS = {"type", "normalized_time", "minutes", "gpu_per_container", "used_gpus"}
TIRESIAS_COLS = {"job_id", "num_gpu", "submit_time", "duration"}


def _f(v, default=0.0) -> float:
    try:
        x = float(v)
        return default if math.isnan(x) else x
    except (TypeError, ValueError):
        return default


def detect_schema(path: str) -> str:
    with open(path) as f:
        header = set(next(csv.reader(f)))
    if LIVE_COLS <= header:
        return "live"
    if TIRESIAS_COLS <= header:
        return "tiresias"
    raise ValueError(f"{path}: unknown trace schema (columns {sorted(header)})")


def read_live_trace(path: str, time_div: float = 10000.0, minutes_scale: float = 1.0,
                    max_jobs: int = 0) -> List[JobSpec]:
    rows = []
    with open(path) as f:
        for i, r in enumerate(csv.DictReader(f)):
            if r.get("type", "noninteractive") != "noninteractive":
                continue
            vals = [r.get(k, "") for k in ("normalized_time", "minutes", "gpu_per_container", "used_gpus",
                                           "gpu_utilization_avg", "gpu_utilization_max", "memory_avg",
                                           "memory_max")]
            if any(v is None or v == "" or (isinstance(v, str) and v.lower() == "nan") for v in vals):
                continue   # reference drops NaN rows (job_generator.py:186)
            rows.append((i, r))
    if not rows:
        return []
    t0 = min(_f(r["normalized_time"]) for _, r in rows)
    specs = []
    for i, r in rows:
        used = max(1, int(_f(r["used_gpus"], 1)))
        gpc = max(1, int(_f(r["gpu_per_container"], 1)))
        gpc = min(gpc, used)
        specs.append(JobSpec(
            job_id=str(r.get("job_id") or i),
            submit_time=(_f(r["normalized_time"]) - t0) / time_div,
            duration=_f(r["minutes"]) * minutes_scale,
            num_gpu=used, gpu_per_worker=gpc,
            model=r.get("model_name", "") or "",
            gpu_util_avg=_f(r.get("gpu_utilization_avg")),
            gpu_util_max=_f(r.get("gpu_utilization_max")),
            gpu_mem_avg=_f(r.get("memory_avg")) / 2 ** 20,
            gpu_mem_max=_f(r.get("memory_max")) / 2 ** 20,
        ))
    specs.sort(key=lambda s: (s.submit_time, _order_key(s.job_id)))
    return specs[:max_jobs] if max_jobs else specs


def read_tiresias_trace(path: str, time_unit: float = 1.0, duration_scale: float = 1.0,
                        max_jobs: int = 0) -> List[JobSpec]:
    specs = []
    with open(path) as f:
        for r in csv.DictReader(f, delimiter="," if not path.endswith(".txt") else " "):
            specs.append(JobSpec(
                job_id=str(r["job_id"]),
                submit_time=_f(r["submit_time"]) * time_unit,
                duration=_f(r["duration"]) * duration_scale,
                num_gpu=max(1, int(_f(r["num_gpu"], 1))),
                model=r.get("model_name", "") or "",
                iterations=int(_f(r.get("iterations"), 0)),
                interval=_f(r.get("interval"), 0),
                gpu_util_avg=_f(r.get("gpu_utilization_avg"), 0),
                gpu_util_max=_f(r.get("gpu_utilization_max"), 0),
                gpu_mem_avg=_f(r.get("memory_avg"), 0),
                gpu_mem_max=_f(r.get("memory_max"), 0),
            ))
    specs.sort(key=lambda s: (s.submit_time, _order_key(s.job_id)))
    return specs[:max_jobs] if max_jobs else specs


def read_trace(path: str, **kw) -> List[JobSpec]:
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    sch = detect_schema(path)
    if sch == "live":
        return read_live_trace(path, **{k: v for k, v in kw.items()
                                        if k in ("time_div", "minutes_scale", "max_jobs")})
    return read_tiresias_trace(path, **{k: v for k, v in kw.items()
                                        if k in ("time_unit", "duration_scale", "max_jobs")})


def read_duration_prior(path: str) -> List[float]:
    with open(path) as f:
        return sorted(_f(r["duration"]) for r in csv.DictReader(f))


def _order_key(job_id: str):
    try:
        return (0, int(job_id), "")
    except ValueError:
        return (1, 0, job_id)


class StreamingReader:
    """Releases trace rows whose submit_time <= t (replaces the reference's
    per-tick pandas mask, job_generator.py:198-207)."""

    def __init__(self, specs: Iterable[JobSpec]):
        self.specs = sorted(specs, key=lambda s: s.submit_time)
        self.cursor = 0

    def release(self, t: float) -> List[JobSpec]:
        out = []
        while self.cursor < len(self.specs) and self.specs[self.cursor].submit_time <= t:
            out.append(self.specs[self.cursor])
            self.cursor += 1
        return out

    def add(self, spec: JobSpec) -> None:
        """Online submission: insert among the not-yet-released rows, in
        submit-time order (a spec dated in the past is released next)."""
        import bisect

        keys = [s.submit_time for s in self.specs[self.cursor:]]
        i = self.cursor + bisect.bisect_right(keys, spec.submit_time)
        self.specs.insert(i, spec)

    def next_time(self) -> float:
        return self.specs[self.cursor].submit_time if self.cursor < len(self.specs) else float("inf")

    def remaining(self) -> int:
        return len(self.specs) - self.cursor


def write_tiresias_trace(path: str, specs: List[JobSpec]) -> None:
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["job_id", "num_gpu", "submit_time", "iterations", "model_name", "duration", "interval",
                    "gpu_utilization_avg", "gpu_utilization_max", "memory_avg", "memory_max"])
        for s in specs:
            w.writerow([s.job_id, s.num_gpu, f"{s.submit_time:.6f}", s.iterations, s.model,
                        f"{s.duration:.6f}", f"{s.interval:.6f}", s.gpu_util_avg, s.gpu_util_max,
                        s.gpu_mem_avg, s.gpu_mem_max])


def write_live_trace(path: str, specs: List[JobSpec], time_div: float = 10000.0) -> None:
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["job_id", "type", "normalized_time", "minutes", "gpu_per_container", "used_gpus",
                    "gpu_utilization_avg", "gpu_utilization_max", "memory_avg", "memory_max", "model_name"])
        for s in specs:
            w.writerow([s.job_id, "noninteractive", s.submit_time * time_div, s.duration,
                        s.gpu_per_worker, s.num_gpu, s.gpu_util_avg, s.gpu_util_max,
                        s.gpu_mem_avg * 2 ** 20, s.gpu_mem_max * 2 ** 20, s.model])
