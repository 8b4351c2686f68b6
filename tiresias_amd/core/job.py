"""Job / Task data model and per-job state machine.

Mirrors the reference's gang-of-tasks model (``/root/reference/core/jobs/
job.py:6-201``: a job of ``total_gpus // gpu_p_worker`` workers named
``worker{i}``, 12 CPUs / 60 GB per task, runs only when *all* tasks run) and
the legacy Tiresias dict-job fields (``run_sim.py`` executed_time,
last_pending_time, q_id, preempt/resume/promote counters), as one explicit
state machine:

    SUBMITTED --arrive--> PENDING --start--> RUNNING --finish--> FINISHED
                             ^                  |
                             +----preempt-------+

Time is float "service units" (seconds for the event engine, ticks for the
reference-compatible tick engine). ``progress`` counts ideal work done; a
job finishes when progress >= duration. ``rate`` (<= 1) models network /
interference slowdowns, ``restore_left`` the checkpoint-restore stall that is
charged after a resume.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple


class JobState(enum.Enum):
    SUBMITTED = "SUBMITTED"
    PENDING = "PENDING"
    RUNNING = "RUNNING"
    FINISHED = "FINISHED"
    FAILED = "FAILED"


@dataclass
class JobSpec:
    """Static description of a job (one trace row)."""
    job_id: str
    submit_time: float
    duration: float                  # service time when placed consolidated, undisturbed
    num_gpu: int
    gpu_per_worker: int = 1
    model: str = ""
    iterations: int = 0
    interval: float = 0.0
    gpu_util_avg: float = 0.0        # percent
    gpu_util_max: float = 0.0
    gpu_mem_avg: float = 0.0         # MiB
    gpu_mem_max: float = 0.0
    cpu_per_task: int = 12           # reference job.py:103
    mem_per_task: int = 60           # reference job.py:104
    user: str = ""

    @property
    def num_workers(self) -> int:
        return max(1, self.num_gpu // max(1, self.gpu_per_worker))


@dataclass
class Task:
    job_id: str
    task_id: str
    index: int
    gpu: int
    cpu: int
    mem: int
    gpu_util_avg: float
    gpu_util_max: float
    gpu_mem_avg: float
    gpu_mem_max: float
    node_id: Optional[str] = None
    devices: Tuple[int, ...] = ()


@dataclass
class Job:
    spec: JobSpec
    state: JobState = JobState.SUBMITTED
    progress: float = 0.0            # ideal work done
    executed: float = 0.0            # service received since last starvation promotion
    total_executed: float = 0.0      # total wall time spent RUNNING
    pending_time: float = 0.0        # total time spent PENDING
    last_pending_time: float = 0.0   # pending time since the job last ran (starvation)
    queue: int = 0
    rank: float = 0.0                # gittins index / policy-specific key
    start_time: Optional[float] = None
    end_time: Optional[float] = None
    last_check: float = 0.0
    preempt_count: int = 0
    resume_count: int = 0
    promote_count: int = 0
    migration_count: int = 0
    rate: float = 1.0
    restore_left: float = 0.0
    ckpt_bytes: float = 0.0
    overhead_time: float = 0.0       # checkpoint/restore time charged
    allocation: Optional[Dict[str, List[int]]] = None   # node_id -> device ids
    allocation_prev: Optional[Dict[str, List[int]]] = None
    tasks: List[Task] = field(default_factory=list)
    credit_key: float = 0.0          # horus+ cluster id etc.
    interfered: bool = False
    last_placement_nodes: int = 0
    extra: Dict = field(default_factory=dict)

    def __post_init__(self):
        if not self.tasks:
            s = self.spec
            self.tasks = [Task(job_id=s.job_id, task_id=f"{s.job_id}_worker{i}", index=i,
                               gpu=max(1, s.gpu_per_worker), cpu=s.cpu_per_task, mem=s.mem_per_task,
                               gpu_util_avg=s.gpu_util_avg, gpu_util_max=s.gpu_util_max,
                               gpu_mem_avg=s.gpu_mem_avg, gpu_mem_max=s.gpu_mem_max)
                          for i in range(s.num_workers)]

    # --------------------------------------------------------------- props
    @property
    def job_id(self) -> str:
        return self.spec.job_id

    @property
    def num_gpu(self) -> int:
        return self.spec.num_gpu

    @property
    def remaining(self) -> float:
        return max(0.0, self.spec.duration - self.progress)

    @property
    def is_running(self) -> bool:
        return self.state == JobState.RUNNING

    @property
    def is_pending(self) -> bool:
        return self.state == JobState.PENDING

    @property
    def done(self) -> bool:
        return self.state in (JobState.FINISHED, JobState.FAILED)

    def attained(self, gputime: bool) -> float:
        """Tiresias attained service: executed time (x #GPUs for 2D-LAS)."""
        return self.executed * self.num_gpu if gputime else self.executed

    @property
    def jct(self) -> Optional[float]:
        if self.end_time is None:
            return None
        return self.end_time - self.spec.submit_time

    # --------------------------------------------------------------- time
    def advance(self, now: float) -> None:
        """Accrue time since last_check according to the current state."""
        dt = now - self.last_check
        if dt < 0:
            raise ValueError(f"time went backwards for job {self.job_id}: {self.last_check} -> {now}")
        if dt == 0:
            return
        if self.state == JobState.RUNNING:
            self.total_executed += dt
            self.executed += dt
            work_dt = dt
            if self.restore_left > 0:
                r = min(self.restore_left, dt)
                self.restore_left -= r
                work_dt -= r
            self.progress = min(self.spec.duration, self.progress + work_dt * self.rate)
        elif self.state == JobState.PENDING:
            self.pending_time += dt
            if self.executed > 0:
                self.last_pending_time += dt
        self.last_check = now

    def time_to_finish(self) -> float:
        if self.state != JobState.RUNNING or self.rate <= 0:
            return float("inf")
        return self.restore_left + self.remaining / self.rate

    # --------------------------------------------------------------- transitions
    def arrive(self, now: float) -> None:
        assert self.state == JobState.SUBMITTED, self.state
        self.state = JobState.PENDING
        self.last_check = now
        self.queue = 0

    def start(self, now: float, allocation: Dict[str, List[int]], rate: float = 1.0,
              restore_cost: float = 0.0) -> None:
        assert self.state == JobState.PENDING, (self.job_id, self.state)
        if self.start_time is None:
            self.start_time = now
        elif self.allocation_prev is not None and self.allocation_prev != allocation:
            self.migration_count += 1
        self.state = JobState.RUNNING
        self.allocation = allocation
        self.rate = rate
        self.resume_count += 1
        # stall before progress resumes: restore + the save of the last preemption
        self.restore_left = restore_cost + self.extra.pop("pending_ckpt", 0.0)
        self.overhead_time += restore_cost
        # last_pending_time is NOT reset on resume: like the reference
        # (run_sim.py:767-778) it accumulates every pending stretch since the
        # job first ran and is cleared only by a starvation promotion
        self.last_check = now

    def preempt(self, now: float, ckpt_cost: float = 0.0, ckpt_bytes: float = 0.0) -> None:
        assert self.state == JobState.RUNNING, (self.job_id, self.state)
        self.state = JobState.PENDING
        self.allocation_prev = self.allocation
        self.allocation = None
        self.preempt_count += 1
        # the checkpoint save is charged as lost progress time on resume
        self.restore_left = 0.0
        self.extra["pending_ckpt"] = self.extra.get("pending_ckpt", 0.0) + ckpt_cost
        self.overhead_time += ckpt_cost
        self.ckpt_bytes += ckpt_bytes
        self.last_check = now

    def finish(self, now: float) -> None:
        assert self.state == JobState.RUNNING
        self.state = JobState.FINISHED
        self.end_time = now
        self.allocation_prev = self.allocation
        self.allocation = None
        self.last_check = now
