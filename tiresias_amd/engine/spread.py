"""Wait-vs-spread advice for the skew-aware placement.

Tiresias (NSDI'19 §4.3) consolidates only placement-SENSITIVE jobs; the
others may take fragments across nodes. Spreading is not free, though: a
gang over k > 1 nodes runs its all-reduce over the inter-node link, so it
progresses at a rate r_k < 1 (measured 2-node slowdown ring-scaled to k
nodes, else the analytic all-reduce, ``cluster/network.py``). On the mixed
ResNet-50 / VGG-16 scenario (profiles/r3/scenarios.md) that made
"fragments first" lose to consolidate-always.

``SpreadAdvisor`` decides, for an insensitive job that has no consolidated
block free, whether spreading NOW beats WAITING for one:

    spread  iff  E[wait for a consolidated block]  >  (1/r_k - 1/r_min) x E[remaining wall time]

Both expectations are non-clairvoyant, like Tiresias itself: a job's
remaining service is E[S - a | S > a] over the service-time history (the
Gittins prior; learned from finished jobs when there is none) given its
attained service a, divided by its GPUs (and its current rate). The wait
for a block is the time until enough running jobs on one node (or on enough
whole nodes, for gangs wider than a node) are expected to finish. Queued
jobs that might claim the block first are ignored (an optimistic wait: it
errs toward consolidating). Under spread_rule ``price`` the spread is also
charged for the queued gangs whose own consolidated block its fragments
delay (``fragment_cost``). The reference has no such rule: its live
``yarn`` path always consolidates (``core/scheduling/algorithm.py:394-415``)
and the model-skew data (``core/models.py:8-26``) is never used.
"""
from __future__ import annotations

import bisect
import math
from typing import Callable, List, Optional


class ServiceEstimate:
    """E[remaining service | attained a] from a sample of job services
    (GPU-seconds), with prefix sums: O(log n) per query."""

    def __init__(self, samples: Optional[List[float]] = None):
        self._d: List[float] = []
        self._pre: List[float] = [0.0]
        self._raw: List[float] = []
        self._next = 0
        if samples:
            self._raw = [float(x) for x in samples]
            self._build()

    def _build(self) -> None:
        self._d = sorted(self._raw)
        self._pre = [0.0]
        for x in self._d:
            self._pre.append(self._pre[-1] + x)
        self._next = max(len(self._d) + 1, int(len(self._d) * 1.1))

    def add(self, s: float) -> None:
        self._raw.append(float(s))
        if len(self._raw) >= self._next:
            self._build()

    def __len__(self) -> int:
        return len(self._d)

    def remaining(self, a: float) -> Optional[float]:
        """Mean of (S - a) over the samples S > a; None without samples. A
        job that outlived every sample is expected to need its attained
        service again (the heavy-tail rule of thumb)."""
        n = len(self._d)
        if n == 0:
            return None
        i = bisect.bisect_right(self._d, a)
        alive = n - i
        if alive == 0:
            return max(a, self._pre[n] / n)
        return (self._pre[n] - self._pre[i]) / alive - a


class SpreadAdvisor:
    """Set on the placement by the engine (``Simulator``); see module doc.

    ``remaining_wall(job)``: expected wall seconds a RUNNING or pending job
    still needs; ``spread_rate(job, k)``: its progress rate over k nodes."""

    def __init__(self, remaining_wall: Callable, spread_rate: Callable, price_fragments: bool = False):
        self.remaining_wall = remaining_wall
        self.spread_rate = spread_rate
        # spread_rule "price": also charge the spread for the queued gangs
        # whose consolidated block it delays (fragment_cost)
        self.price_fragments = price_fragments
        self.decisions = {"spread": 0, "wait": 0}

    def wait_for_block(self, cluster, job, jobs_by_id, gpn: int, min_nodes: int) -> float:
        """Expected seconds until ``job`` could be placed on ``min_nodes``
        nodes (one node with job.num_gpu free GPUs, or min_nodes whole free
        nodes), from the running jobs' expected remaining times."""
        per_node = {nid: [] for nid in cluster.nodes}
        for jid, parts in cluster.placed.items():
            j = jobs_by_id.get(jid)
            if j is None:
                continue
            rem = self.remaining_wall(j)
            for nid, devs in parts:
                if nid in per_node:
                    per_node[nid].append((rem, len(devs)))
        need_whole = job.num_gpu > gpn
        times = []
        for nid, node in cluster.nodes.items():
            free = node.num_free_gpus()
            cap = node.gpu_count - sum(1 for d in node.devices if getattr(d, "failed", False))
            if need_whole:
                if cap < node.gpu_count:
                    continue
                times.append(max([r for r, _ in per_node[nid]], default=0.0))
                continue
            if cap < job.num_gpu:
                continue
            t = 0.0
            for rem, n in sorted(per_node[nid]):
                if free >= job.num_gpu:
                    break
                free += n
                t = rem
            if free >= job.num_gpu:
                times.append(t)
        if need_whole:
            times.sort()
            return times[min_nodes - 1] if len(times) >= min_nodes else math.inf
        return min(times, default=math.inf)

    def fragment_cost(self, cluster, job, jobs_by_id, gpn: int, hold_s: float) -> float:
        """What a spread of ``job`` costs the QUEUED gangs, in ``job``'s own
        seconds: the spread holds node fragments for ``hold_s`` (its expected
        wall time at the spread rate); a pending gang q whose consolidated
        block would otherwise free up after w_q < hold_s waits hold_s - w_q
        longer, weighted by its GPUs over the job's. Every queued gang is
        assumed to want the touched nodes (a conservative charge). The terms
        are summed in ascending order, as the native core does, so both
        engines take the same decision (tests/test_sched_core.py)."""
        terms = []
        for q in jobs_by_id.values():
            if q is job or not q.is_pending or q.num_gpu < 2:
                continue
            w = self.wait_for_block(cluster, q, jobs_by_id, gpn, max(1, math.ceil(q.num_gpu / gpn)))
            if w < hold_s:
                terms.append((hold_s - w) * q.num_gpu / max(1, job.num_gpu))
        return sum(sorted(terms))

    def should_spread(self, cluster, job, jobs_by_id, k: int, gpn: int, min_nodes: int, count: bool = True) -> bool:
        r_k = self.spread_rate(job, k)
        r_min = self.spread_rate(job, min_nodes)
        rem = self.remaining_wall(job)
        if rem is None or r_k <= 0:
            ok = True                      # no history yet: the skew-aware default
        else:
            penalty = (1.0 / r_k - 1.0 / max(r_min, 1e-9)) * rem
            if self.price_fragments:
                penalty += self.fragment_cost(cluster, job, jobs_by_id, gpn, rem / r_k)
            ok = self.wait_for_block(cluster, job, jobs_by_id, gpn, min_nodes) > penalty
        if count:
            self.decisions["spread" if ok else "wait"] += 1
        return ok
