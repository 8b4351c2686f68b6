"""The live reference's policies: Horus, Horus+ and Gandiva
(``/root/reference/core/scheduling/algorithm.py:189-296, 418-442``,
``core/jobs/job_queue_manager.py``, ``core/jobs/utils.py``).

* ``horus``: non-preemptive; pending jobs ordered lowest average GPU
  utilisation first (the reference heap, ``base_factory.py:2-14``), the first
  ``lookahead`` (k=5) are tried in order and the ones that fit start.
* ``horus+``: pending jobs are clustered into ``num_queue`` queues by k-means
  over job features (#tasks, util avg/max, GPUs per worker, GPUs, mem
  avg/max; L1 distance, medoid centroids, ``utils.py:4-67``) — SEEDED here
  (defect D10) and re-clustered only when the pending set changes, not on every
  insert; each pick comes from the queue with the highest credit
  (median pending time x length, or length when the median is < 1,
  ``job_queue_manager.py:103-127``).
* ``gandiva``: FIFO order + Gandiva (co-locating) placement + time slicing:
  whenever jobs are waiting, a running job is preempted at every multiple of
  the quantum of its run time (``time_slice_check`` :418-438).
* migration (``schedule.py:62-93``, defect D7: never fires in the
  reference) lives in the engine (``engine/sim.py::_migrate``).
"""
from __future__ import annotations

import heapq
import random
from statistics import median
from typing import List, Optional, Sequence

from ..core.job import Job
from .base import INF, Policy, register, submit_key


def _features(j: Job) -> List[float]:
    s = j.spec
    return [len(j.tasks), s.gpu_util_avg, s.gpu_per_worker, s.num_gpu, s.gpu_util_max,
            s.gpu_mem_avg, s.gpu_mem_max]


def _l1(a: Sequence[float], b: Sequence[float]) -> float:
    return sum(abs(x - y) for x, y in zip(a, b))


def kmeans_jobs(jobs: List[Job], k: int, rng: random.Random, max_iter: int = 1000):
    """k-medoids-style clustering on job features (seeded)."""
    if not jobs:
        return [], [], 0.0
    k = max(1, min(k, len(jobs)))
    feats = [_features(j) for j in jobs]
    cent = [feats[i] for i in rng.sample(range(len(jobs)), k)]
    assign = [-1] * len(jobs)
    for _ in range(max_iter):
        new = [min(range(k), key=lambda c: (_l1(f, cent[c]), c)) for f in feats]
        if new == assign:
            break
        assign = new
        for c in range(k):
            members = [feats[i] for i in range(len(jobs)) if assign[i] == c]
            if not members:
                cent[c] = feats[rng.randrange(len(jobs))]
                continue
            mean = [sum(col) / len(members) for col in zip(*members)]
            cent[c] = min(members, key=lambda m: _l1(m, mean))
    loss = sum(_l1(feats[i], cent[assign[i]]) for i in range(len(jobs)))
    return cent, assign, loss


class _RefItem:
    """A queued job as the reference's heap sees it
    (``core/jobs/base_factory.py:2-14`` CompareAbleByUtilization): lower
    average utilisation first, and ``<`` is False between equal (or zero)
    utilisations -- so heapq's sift, not arrival order, decides among ties."""
    __slots__ = ("job",)

    def __init__(self, job: Job):
        self.job = job

    def __lt__(self, other: "_RefItem") -> bool:
        a = self.job.spec.gpu_util_avg
        return bool(a) and a < other.job.spec.gpu_util_avg


@register("horus")
class Horus(Policy):
    """Event engine: pending jobs in (utilisation, arrival) order. Under the
    reference-compatible tick engine (``cfg.engine == "tick"``) the queue is
    the reference's own heap operation for operation (``schedule_horus``,
    ``algorithm.py:204-238``): every tick pops min(k, queued) jobs, the
    engine places the first that fits, and the rest are pushed back in
    look-ahead order -- which reorders equal-utilisation jobs exactly as the
    reference does (pinned by tests/test_ref_parity.py's hplus_queue trace)."""
    default_placement = "horus"

    def __init__(self, cfg=None, prior=None, rng=None):
        super().__init__(cfg, prior, rng)
        self.lookahead = int(getattr(cfg, "lookahead", 5) or 5)
        self.ref_heap = getattr(cfg, "engine", "event") == "tick"
        self._heap: List[_RefItem] = []
        self._look: List[Job] = []

    def on_arrival(self, job, now):
        super().on_arrival(job, now)
        if self.ref_heap:
            heapq.heappush(self._heap, _RefItem(job))

    def order(self, active, now):
        if self.ref_heap:
            n = min(self.lookahead, len(self._heap))
            self._look = [heapq.heappop(self._heap).job for _ in range(n)]
            return list(self._look)
        return sorted((j for j in active if j.is_pending),
                      key=lambda j: (j.spec.gpu_util_avg, submit_key(j)))

    def after_schedule(self, active, now):
        if self.ref_heap:
            # the look-ahead jobs that did not start go back (jobs_manager.insert)
            for j in self._look:
                if j.is_pending:
                    heapq.heappush(self._heap, _RefItem(j))
            self._look = []


@register("horus+")
class HorusPlus(Horus):
    def __init__(self, cfg=None, prior=None, rng=None):
        super().__init__(cfg, prior, rng)
        self.k = max(1, int(getattr(cfg, "num_queue", 3) or 3))
        self.rng = rng or random.Random(getattr(cfg, "seed", 0) or 0)
        self._key = None
        self._assign = {}
        self._queues: List[List[_RefItem]] = [[] for _ in range(self.k)]
        self._batch: List[Job] = []

    def credits(self, queues: List[List[Job]]) -> List[float]:
        out = []
        for q in queues:
            if not q:
                out.append(0.0)
                continue
            m = max(0.0, median(j.pending_time for j in q))
            out.append(len(q) if m < 1 else m * len(q))
        return out

    # ---- reference-compatible tick engine: num_queue heaps; every tick's
    # insert (gen_jobs -> jobs_manager.insert, with or without arrivals) pops
    # ALL queued jobs (heap order, queue by queue) and re-inserts them + the
    # batch at their k-means queue (jobs_manager.py:115-140); each
    # of the tick's look-ahead pops takes the queue with the highest credit
    # (schedule_horus_plus, algorithm.py:240-288); non-starters go back to
    # their queue
    def on_arrival(self, job, now):
        Policy.on_arrival(self, job, now)
        if self.ref_heap:
            self._batch.append(job)

    def _ref_insert_batch(self) -> None:
        # every tick, even with no arrival: gen_jobs always calls insert(),
        # which for horus+ pops and re-clusters the whole queue
        queued = []
        for q in self._queues:
            while q:
                queued.append(heapq.heappop(q).job)
        jobs = queued + self._batch
        self._batch = []
        _, assign, _ = kmeans_jobs(jobs, self.k, self.rng)
        for j, qi in zip(jobs, assign):
            heapq.heappush(self._queues[qi], _RefItem(j))
            j.queue = qi

    def _ref_credits(self) -> List[float]:
        return self.credits([[it.job for it in q] for q in self._queues])

    def order(self, active, now):
        if self.ref_heap:
            self._ref_insert_batch()
            n = min(self.lookahead, sum(len(q) for q in self._queues))
            self._look = []
            for _ in range(n):
                cr = self._ref_credits()
                qi = max(range(self.k), key=lambda i: (cr[i], -i))     # np.argmax: first maximum
                self._look.append((heapq.heappop(self._queues[qi]).job, qi))
            return [j for j, _ in self._look]
        pend = sorted((j for j in active if j.is_pending), key=submit_key)
        key = tuple(j.job_id for j in pend)
        if key != self._key:
            _, assign, _ = kmeans_jobs(pend, self.k, self.rng)
            self._assign = {j.job_id: a for j, a in zip(pend, assign)}
            self._key = key
        queues: List[List[Job]] = [[] for _ in range(self.k)]
        for j in pend:
            queues[self._assign.get(j.job_id, 0)].append(j)
        for q in queues:
            q.sort(key=lambda j: (j.spec.gpu_util_avg, submit_key(j)))
        out = []
        while any(queues):
            cr = self.credits(queues)
            qi = max(range(self.k), key=lambda i: (cr[i], -i))
            out.append(queues[qi].pop(0))
        return out

    def after_schedule(self, active, now):
        if self.ref_heap:
            for j, qi in self._look:
                if j.is_pending:
                    heapq.heappush(self._queues[qi], _RefItem(j))
            self._look = []


@register("gandiva")
class Gandiva(Policy):
    blocking = True
    default_placement = "gandiva"

    def __init__(self, cfg=None, prior=None, rng=None):
        super().__init__(cfg, prior, rng)
        self.quantum = float(getattr(cfg, "timeslice", 100.0) or 100.0)

    def order(self, active, now):
        return sorted((j for j in active if j.is_pending),
                      key=lambda j: (j.extra.get("requeue", 0.0), submit_key(j)))

    def _slice_end(self, j: Job) -> float:
        return j.extra.get("run_start", j.last_check) + self.quantum

    def preempt_now(self, active, now):
        if not any(j.is_pending for j in active):
            return []
        out = [j for j in active if j.is_running and self._slice_end(j) <= now + 1e-9]
        for j in out:
            j.extra["requeue"] = now
        return out

    def next_event(self, active, now):
        if not any(j.is_pending for j in active):
            return INF
        ends = [self._slice_end(j) for j in active if j.is_running]
        return min(ends) if ends else INF
