"""The live reference's policies: Horus, Horus+ and Gandiva
(``/root/reference/core/scheduling/algorithm.py:189-296, 418-442``,
``core/jobs/job_queue_manager.py``, ``core/jobs/utils.py``).

* ``horus``: non-preemptive; pending jobs ordered lowest average GPU
  utilisation first (the reference heap, ``base_factory.py:2-14``), the first
  ``lookahead`` (k=5) are tried in order and the ones that fit start.
* ``horus+``: pending jobs are clustered into ``num_queue`` queues by the
  reference's k-means over job features (#tasks, util avg/max, GPUs per
  worker, GPUs, mem avg/max; L1 distance, centroids re-picked by the scalar
  feature-sum score, ``utils.py:4-67``) — SEEDED here (defect D10) with a
  numpy RandomState, and pinned against the executed reference
  (``tests/test_ref_parity.py::test_kmeans_matches_reference``); the event
  engine re-clusters only when the pending set changes, the tick engine on
  every insert as the reference does; each pick comes from the queue with the highest credit
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


def kmeans_jobs(jobs: List[Job], k: int, rng, max_iter: int = 1000):
    """The reference's horus+ k-means (``core/jobs/utils.py:36-67``),
    SEEDED (defect D10), operation for operation so that the same
    ``numpy.random.RandomState`` stream gives the same clusters:

    * init: ``k`` centroid jobs drawn WITH replacement,
      ``rng.randint(len(jobs), size=k)`` (:39); duplicates are allowed;
    * assignment: L1 feature distance (``job_dist`` :4-12), first minimum
      (``np.argmin``);
    * update: a cluster's new centroid is the member whose SCALAR score
      (``transform_to_dist`` :14-22, the feature sum) is closest to the
      int-truncated mean score, first minimum (``get_closest`` :24-34,
      ``np.mean(...).astype(int)`` :58); an empty cluster re-draws a random
      job (``rng.choice(len(jobs))`` :62);
    * the loop runs while the assignment changed (or on the first pass) and
      updates the centroids in every pass, the converged one included, as
      the reference's does (:45-62) -- the RNG stream stays in step.

    ``rng``: a ``numpy.random.RandomState`` (a ``random.Random`` is mapped
    onto one seeded from it). Returns (centroid indices, assignment, loss)."""
    import numpy as np

    if not jobs:
        return [], [], 0.0
    if not isinstance(rng, np.random.RandomState):
        rng = np.random.RandomState(rng.randrange(1 << 31) if hasattr(rng, "randrange") else int(rng))
    k = max(1, int(k))
    n = len(jobs)
    feats = [_features(j) for j in jobs]
    score = [float(sum(f)) for f in feats]
    cent = [int(i) for i in rng.randint(n, size=k)]
    new: List = [None] * n
    old: List = [None] * n
    it = 0
    while it < max_iter and (new != old or it == 0):
        old = list(new)
        it += 1
        for i in range(n):
            d = [_l1(feats[i], feats[cent[c]]) for c in range(k)]
            new[i] = min(range(k), key=lambda c: (d[c], c))
        for c in range(k):
            members = [i for i in range(n) if new[i] == c]
            if members:
                mean = int(np.mean([score[i] for i in members], axis=0).astype(int))
                best, best_d = None, 99999999999
                for i in members:                    # get_closest: strict <, first minimum
                    t = abs(score[i] - mean)
                    if t < best_d:
                        best, best_d = i, t
                cent[c] = best
            else:
                cent[c] = int(rng.choice(n))
    loss = sum(_l1(feats[i], feats[cent[new[i]]]) for i in range(n))
    return cent, list(new), loss


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
        # the reference draws its k-means init from numpy's global stream:
        # a seeded RandomState of its own here (D10)
        import numpy as np
        self.rng = np.random.RandomState(int(getattr(cfg, "seed", 0) or 0))
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
