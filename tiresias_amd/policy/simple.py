"""Baseline policies from the legacy Tiresias simulator
(``/root/reference/run_sim.py``): FIFO (``sim_job_events`` :1533-1599), FJF,
SJF (``smallest_first_sim_jobs`` :161-286), SRTF / SRSF / shortest-expected
(``shortest_first_sim_jobs`` :298-430, ``cal_shortest_expected_remaining``
:288-296) and LPJF (``longest_pending_first_sim_jobs`` :1474-1531).

Deviation from the live reference FIFO (defect D8: new batches and
preempted jobs were inserted at the queue HEAD): FIFO here is strict arrival
order.
"""
from __future__ import annotations

import bisect
from typing import List

from ..core.job import Job
from .base import Policy, register, submit_key


@register("fifo")
class FIFO(Policy):
    """Non-preemptive, head-of-line blocking (YARN-CS FIFO baseline)."""
    blocking = True

    def order(self, active, now):
        return sorted((j for j in active if j.is_pending), key=submit_key)


@register("fjf")
class FitJobFirst(FIFO):
    """FIFO order, but any job that fits may start (no head-of-line blocking)."""
    blocking = False


@register("sjf")
class SmallestJobFirst(Policy):
    """Preemptive smallest-GPU-demand first."""
    preemptive = True

    def order(self, active, now):
        return sorted(active, key=lambda j: (j.num_gpu, submit_key(j)))


@register("shortest")
class SRTF(Policy):
    """Preemptive shortest-remaining-time first (oracle: knows durations)."""
    preemptive = True
    gputime = False

    def _key(self, j: Job):
        r = j.remaining
        return r * j.num_gpu if self.gputime else r

    def order(self, active, now):
        return sorted(active, key=lambda j: (self._key(j), submit_key(j)))


@register("shortest-gpu")
class SRSF(SRTF):
    """Preemptive shortest-remaining-GPU-service first (oracle)."""
    gputime = True


@register("shortest-expected")
class ShortestExpected(Policy):
    """Preemptive by expected remaining service E[D - a | D > a] from the
    duration prior (no oracle knowledge of the job's own duration)."""
    preemptive = True

    def __init__(self, cfg=None, prior=None, rng=None):
        super().__init__(cfg, prior, rng)
        self._samples = list(prior or [])
        self._build()

    def _build(self):
        self.data = sorted(self._samples)
        self.suffix = [0.0] * (len(self.data) + 1)
        for i in range(len(self.data) - 1, -1, -1):
            self.suffix[i] = self.suffix[i + 1] + self.data[i]
        self._next_build = max(len(self.data) + 1, int(len(self.data) * 1.1))

    def on_finish(self, job, now):
        if self.prior is None:        # no history file: learn from finished jobs
            self._samples.append(job.total_executed)
            if len(self._samples) >= self._next_build:
                self._build()

    def expected_remaining(self, a: float) -> float:
        if not self.data:
            return 0.0
        i = bisect.bisect_right(self.data, a)
        n = len(self.data) - i
        if n <= 0:
            return 0.0
        return self.suffix[i] / n - a

    def order(self, active, now):
        return sorted(active, key=lambda j: (self.expected_remaining(j.executed), submit_key(j)))


@register("lpjf")
class LongestPendingFirst(Policy):
    """Non-preemptive; the longest-waiting pending job first (blocking)."""
    blocking = True

    def order(self, active, now):
        return sorted((j for j in active if j.is_pending),
                      key=lambda j: (-j.pending_time, submit_key(j)))
