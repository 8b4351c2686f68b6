"""Tiresias' core policies: Discretized 2D-LAS and the Gittins index.

Semantics follow the legacy simulator (``/root/reference/run_sim.py``):

* ``dlas`` / ``dlas-gpu`` (``dlas_sim_jobs`` :663-946): K priority queues
  with demotion thresholds on attained service — executed time, or executed
  time x #GPUs for 2D-LAS. New jobs enter Q0 (:731-733); a job is demoted
  when attained >= limit[q] (:752-758); within a queue jobs run FIFO with
  pending jobs moved behind running ones after every scheduling round
  (:837-847) to avoid thrashing; admission walks Q0..QK-1 and runs every job
  whose GPUs fit (work conserving). Starvation knob: a pending job in Qi>0
  whose pending time since it last ran reaches executed*solve_starvation is
  promoted to Q0 and its executed time reset (:771-778). The engine wakes at
  the next demotion / promotion time (:907-943).
* ``dlas-gpu-gittins`` (:807-809, :948-953): same queues, ordered inside each
  queue by the Gittins index of the job's attained GPU service.
* ``gittins`` (``gittins_sim_jobs`` :955-1202): one queue ordered by Gittins
  index, re-evaluated every ``gittins_delta`` of attained service.
* ``multi-dlas-gpu`` (``multi_dlas_sim_jobs`` :432-661): separate 2D-LAS
  queues per GPU-size class with a GPU reservation per class re-planned every
  ``replan_interval``; leftover GPUs are back-filled in global order.
* ``dlas-gpu-pack`` (:1204-1472): 2D-LAS with GPU sharing (``pack``
  placement).

Gittins index (``cal_r_gittins_index`` :1649-1680): for attained service a and
quantum D, over the prior duration sample,
    P = Pr(S <= a + D | S > a),   E = E[min(S, a + D) - a | S > a],
    G(a) = P / E   (0 beyond the largest sample).
The reference's E sums the raw durations instead of the service still to be
received (min(S, a+D) - a); ``legacy_formula=True`` reproduces that.
"""
from __future__ import annotations

import bisect
import math
from typing import Dict, List, Optional

from ..core.job import Job
from .base import INF, Policy, register, submit_key


class GittinsTable:
    """Gittins index over a service-time sample.

    The sample comes from HISTORY, never from the jobs being scheduled: a
    prior file (``--gittins_prior``, the reference's ``yarn-gput1000.csv``,
    ``run_sim.py:1682-1707``), or -- with no file -- the services of the jobs
    that have FINISHED so far (``add``; online learning, no look-ahead). The
    online table is rebuilt when the sample has grown by 10 % (at least one
    sample), so a 20k-job replay costs O(n log n); the native core
    (``csrc/sched_core/engine.h``) applies the same rule."""

    def __init__(self, durations: List[float], delta: float, legacy_formula: bool = False):
        self.delta = float(delta)
        self.legacy = legacy_formula
        self._samples = [float(d) for d in durations]
        self._next_build = 0
        self._build()

    def _build(self) -> None:
        self.data = sorted(self._samples)
        n = len(self.data)
        self.prefix = [0.0] * (n + 1)
        for i, d in enumerate(self.data):
            self.prefix[i + 1] = self.prefix[i] + d
        self._next_build = max(n + 1, int(n * 1.1))

    def add(self, service: float) -> None:
        self._samples.append(float(service))
        if len(self._samples) >= self._next_build:
            self._build()

    def index(self, a: float) -> float:
        n = len(self.data)
        if n == 0:
            return 0.0
        i = bisect.bisect_right(self.data, a)          # first sample > a
        alive = n - i
        if alive <= 0:
            return 0.0
        j = bisect.bisect_right(self.data, a + self.delta)
        done = j - i                                     # a < S <= a + delta
        P = done / alive
        if self.legacy:
            E = ((self.prefix[j] - self.prefix[i]) + self.delta * (n - j)) / alive
            return P * 1e6 / E if E > 0 else 0.0
        E = ((self.prefix[j] - self.prefix[i]) - a * done + self.delta * (n - j)) / alive
        return P / E if E > 0 else 0.0


def default_limits(num_queue: int, base: float) -> List[float]:
    """K-1 thresholds, exponentially spaced (Tiresias §4.1 uses exponentially
    growing queue thresholds)."""
    return [base * (2 ** i) for i in range(max(0, num_queue - 1))]


@register("dlas", "dlas-gpu", "dlas-gpu-gittins", "dlas-gpu-pack")
class DLAS(Policy):
    preemptive = True

    def __init__(self, cfg=None, prior=None, rng=None):
        super().__init__(cfg, prior, rng)
        nq = max(1, getattr(cfg, "num_queue", 2) or 2)
        limits = list(getattr(cfg, "queue_limits", []) or [])
        if not limits:
            limits = default_limits(nq if nq > 1 else 2, 3600.0)
        self.limits = sorted(float(x) for x in limits)
        self.nq = len(self.limits) + 1
        self.starve = float(getattr(cfg, "solve_starvation", 0.0) or 0.0)
        self.gittins: Optional[GittinsTable] = None
        self._gputime = True

    @property
    def gputime(self) -> bool:
        return self.name != "dlas"

    def _ensure_gittins(self):
        if self.name == "dlas-gpu-gittins" and self.gittins is None:
            delta = getattr(self.cfg, "gittins_delta", 3250.0) or 3250.0
            self.gittins = GittinsTable(self.prior or [], delta)

    def on_finish(self, job, now):
        if self.prior is None:                  # online prior: learn from finished jobs
            self._ensure_gittins()
            if self.gittins is not None:
                self.gittins.add(job.total_executed * job.num_gpu)

    def _enter(self, j: Job, q: int):
        j.queue = q
        j.extra["seq"] = self.next_seq()

    def on_arrival(self, job, now):
        self._enter(job, 0)

    def update(self, active, now):
        self._ensure_gittins()
        g = self.gputime
        # the event clock's relative tolerance: a threshold whose remaining
        # time rounds to "now" fires now (else the engine would stall on it)
        tol = 1e-9 * max(1.0, now)
        for j in active:
            a = j.attained(g)
            if j.is_running:
                while j.queue < self.nq - 1 and a >= self.limits[j.queue] - tol * (j.num_gpu if g else 1):
                    self._enter(j, j.queue + 1)
            elif (self.starve > 0 and j.is_pending and j.queue > 0 and j.executed > 0
                  and j.last_pending_time >= j.executed * self.starve - tol):
                j.executed = 0.0
                j.last_pending_time = 0.0
                j.promote_count += 1
                self._enter(j, 0)
            if self.gittins is not None:
                j.rank = self.gittins.index(j.attained(g))

    def _key(self, j: Job):
        if self.gittins is not None:
            # reference :807-809 re-sorts each queue by rank every event; ties
            # keep running jobs first (no thrash between equal-rank jobs)
            return (j.queue, -j.rank, 0 if j.is_running else 1, j.extra.get("seq", 0))
        # FIFO by queue-entry order only: a job demoted into Qi gets a new seq
        # and so queues BEHIND the jobs already pending in Qi (reference
        # :752-757 appends it to the tail); pending jobs are moved behind the
        # running ones by after_schedule (:837-847)
        return (j.queue, j.extra.get("seq", 0))

    def order(self, active, now):
        return sorted(active, key=self._key)

    def after_schedule(self, active, now):
        # pending jobs move behind running ones inside each queue (reference :837-847)
        for j in sorted((j for j in active if j.is_pending), key=lambda j: (j.queue, j.extra.get("seq", 0))):
            j.extra["seq"] = self.next_seq()

    def next_event(self, active, now):
        t = INF
        g = self.gputime
        for j in active:
            if j.is_running and j.queue < self.nq - 1:
                left = self.limits[j.queue] - j.attained(g)
                t = min(t, now + max(0.0, left) / (j.num_gpu if g else 1))
            elif (self.starve > 0 and j.is_pending and j.queue > 0 and j.executed > 0):
                left = j.executed * self.starve - j.last_pending_time
                if left > 0:
                    t = min(t, now + left)
            if self.gittins is not None and j.is_running:
                t = min(t, now + _quantum_wait(j.attained(g), self.gittins.delta, j.num_gpu if g else 1, now))
        return t


def _quantum_wait(a: float, d: float, div: float, now: float) -> float:
    """Wall seconds until attained service ``a`` (accruing at ``div`` per
    second) reaches the next Gittins quantum boundary. A boundary closer than
    the event clock's tolerance (1e-9 x now: the engine snaps such events to
    now, where no service accrues) counts as reached -- else a long replay
    with a wide gang stalls on it (csrc/sched_core/engine.h::quantum_wait is
    the same rule)."""
    w = ((math.floor(a / d + 1e-6) + 1) * d - a) / div
    if w <= 1e-9 * max(1.0, now):
        w += d / div
    return w


@register("gittins")
class Gittins(Policy):
    """Single-queue Gittins-index scheduling on attained GPU service."""
    preemptive = True

    def __init__(self, cfg=None, prior=None, rng=None):
        super().__init__(cfg, prior, rng)
        self.delta = float(getattr(cfg, "gittins_delta", 3250.0) or 3250.0)
        self.table = GittinsTable(prior or [], self.delta)

    def on_finish(self, job, now):
        if self.prior is None:                  # online prior: learn from finished jobs
            self.table.add(job.total_executed * job.num_gpu)

    def update(self, active, now):
        for j in active:
            j.rank = self.table.index(j.attained(True))

    def order(self, active, now):
        return sorted(active, key=lambda j: (-j.rank, 0 if j.is_running else 1, submit_key(j)))

    def next_event(self, active, now):
        t = INF
        for j in active:
            if j.is_running:
                t = min(t, now + _quantum_wait(j.attained(True), self.delta, j.num_gpu, now))
        return t


@register("multi-dlas-gpu", "multi-dlas")
class MultiDLAS(DLAS):
    """Per-GPU-size-class 2D-LAS with periodic GPU reservations."""

    def __init__(self, cfg=None, prior=None, rng=None):
        super().__init__(cfg, prior, rng)
        self.interval = float(getattr(cfg, "replan_interval", 600.0) or 600.0)
        self.next_replan = 0.0
        self.reserve: Dict[int, int] = {}
        self.total_gpus = None

    @property
    def gputime(self) -> bool:
        return True

    def _replan(self, active, total):
        demand: Dict[int, int] = {}
        for j in active:
            demand[j.num_gpu] = demand.get(j.num_gpu, 0) + j.num_gpu
        tot = sum(demand.values())
        self.reserve = {}
        if tot == 0:
            return
        left = total
        for c in sorted(demand):
            r = int(total * demand[c] / tot)
            r = max(r, c) if left >= c else r
            r = min(r, left)
            self.reserve[c] = r
            left -= r

    def select(self, ordered, free_gpus, now):
        total = free_gpus + sum(j.num_gpu for j in ordered if j.is_running)
        if now >= self.next_replan or self.total_gpus != total:
            self._replan(ordered, total)
            self.total_gpus = total
            while self.next_replan <= now:
                self.next_replan += self.interval
        chosen, used = [], 0
        per_class_used: Dict[int, int] = {}
        for j in ordered:
            c = j.num_gpu
            if per_class_used.get(c, 0) + c <= self.reserve.get(c, 0) and used + c <= total:
                chosen.append(j)
                per_class_used[c] = per_class_used.get(c, 0) + c
                used += c
        for j in ordered:                               # work-conserving back-fill
            if j not in chosen and used + j.num_gpu <= total:
                chosen.append(j)
                used += j.num_gpu
        return chosen

    def next_event(self, active, now):
        return min(super().next_event(active, now), self.next_replan if active else INF)
