"""Legacy Gandiva node-set engine (``--schedule gandiva-ns``).

Reproduces the dead ``gandiva_sim_jobs`` path of the reference
(``run_sim.py:101-158``; ``infra/cluster.py:150-489``), which the live
``gandiva`` policy (``policy/horus.py``) does not cover:

* **node-sets per job size** — nodes are grouped into sets dedicated to one job
  size g in {1, 2, 4, ...}; a set spans ceil(g / gpus_per_node) nodes and has
  ``capacity = nodes * gpus_per_node / g`` slots (``cluster.py:215-227``);
* **placement** — a job goes to the least-utilised set of its class when its
  ``mem_util`` still fits, else a new set is carved from free nodes, else it is
  time-sliced onto the least-utilised existing set; with no set of its class
  and no free node it pends (``cluster.py:166-251``);
* **grow / shrink** — every tick the free nodes are re-divided between classes
  in proportion to their GPU demand (#jobs x g), expanding or dissolving sets
  and re-spreading their jobs (``cluster.py:255-382``);
* **time-slicing** — inside a set the leading jobs whose cumulative
  ``mem_util`` fits run; every ``slice`` seconds those are rotated to the back
  (``cluster.py:386-489``, 60 s);
* fixed ``tick`` (10 s) event loop that also stops at arrivals
  (``run_sim.py:140-156``).

Deliberate differences (documented defects of the reference):
* job sizes that are not a power of two use the next power-of-two class (the
  reference ``exit()``s, ``cluster.py:172-175``);
* a job finishing inside a tick ends at its exact time (the reference rounds
  completion up to the tick), and per-job rows / preemption counts are logged
  (the reference's ``job_complete`` writes only a subset);
* the shrink path cannot dissolve the class's last set while it holds jobs
  (``cluster.py:263-265`` can leave jobs without a set).

``mem_util`` per job: ``one`` (reference live table, ``core/models.py:19``: every
model 1.0 = one slot), ``legacy`` (the commented table, ``core/models.py:18``)
or ``measured`` (``profiler.memory`` estimate of the job's HBM fraction on the
configured GPU).
"""
from __future__ import annotations

import math
import time
from typing import Dict, List, Optional

from ..config import SimConfig
from ..core.job import Job, JobSpec, JobState
from ..metrics.logger import MetricsLogger

LEGACY_MEM_UTIL = {"vgg19": 0.60, "vgg16": 0.55, "vgg11": 0.45, "alexnet": 0.13, "resnet152": 0.85,
                   "resnet101": 0.70, "resnet50": 0.50, "inception4": 0.85, "inception3": 0.80}


def _pow2_class(g: int) -> int:
    return 1 << max(0, math.ceil(math.log2(max(1, g))))


class _NodeSet:
    __slots__ = ("g", "nodes", "capacity", "jobs")

    def __init__(self, g: int, nodes: List[str], gpn: int):
        self.g = g
        self.nodes = nodes
        self.capacity = max(1, int(len(nodes) * gpn / g))
        self.jobs: List[Job] = []

    def util(self, mu) -> float:
        return round(sum(mu(j) for j in self.jobs), 2)


class GandivaNodeSetSim:
    def __init__(self, cfg: SimConfig, specs: List[JobSpec], logger: Optional[MetricsLogger] = None,
                 tick: float = 10.0, slice_s: float = 60.0, mem_util: str = "one"):
        self.cfg = cfg
        self.log = logger or MetricsLogger(None)
        c = cfg.cluster
        self.gpn = c.num_gpu_p_node
        n_nodes = c.num_switch * c.num_node_p_switch
        self.num_gpus = n_nodes * self.gpn
        self.total_nodes = n_nodes
        self.free: List[str] = [str(i + 1) for i in range(n_nodes)]
        self.sets: Dict[int, List[_NodeSet]] = {}
        self.tick, self.slice = float(tick), float(slice_s)
        self.mem_mode = mem_util
        self.jobs: Dict[str, Job] = {}
        self.arrivals = sorted(specs, key=lambda s: (s.submit_time, s.job_id))
        self.pending: List[Job] = []
        self.now = 0.0
        self.wall_s = 0.0

    # ------------------------------------------------------------ helpers
    def _mu(self, j: Job) -> float:
        if self.mem_mode == "legacy":
            return LEGACY_MEM_UTIL.get(j.spec.model, 1.0)
        if self.mem_mode == "measured":
            from ..profiler.memory import estimate_gpu_memory

            return round(estimate_gpu_memory(j.spec.model or "resnet50",
                                             capacity_mb=self.cfg.cluster.gpu_memory_mb)["fraction"], 2)
        return 1.0

    def _nodes_for(self, g: int) -> int:
        return int(math.ceil(g / self.gpn))

    def _sorted(self, g: int) -> List[_NodeSet]:
        lst = self.sets.setdefault(g, [])
        lst.sort(key=lambda ns: ns.util(self._mu))
        return lst

    def _new_set(self, g: int) -> Optional[_NodeSet]:
        k = self._nodes_for(g)
        if k > len(self.free):
            return None
        ns = _NodeSet(g, [self.free.pop(0) for _ in range(k)], self.gpn)
        self.sets.setdefault(g, []).append(ns)
        return ns

    def _place(self, j: Job) -> bool:
        g = _pow2_class(j.num_gpu)
        lst = self._sorted(g)
        # strict '<' as in the reference (cluster.py:204): a 4-slot set takes 3 one-slot jobs
        # before a new set is opened; the 4th slot is used by time-slicing / re-spreading
        if lst and lst[0].util(self._mu) + self._mu(j) < lst[0].capacity - 1e-9:
            lst[0].jobs.append(j)
            return True
        ns = self._new_set(g)
        if ns is not None:
            ns.jobs.append(j)
            return True
        if lst:                                   # time-slice onto the least-loaded set
            lst[0].jobs.append(j)
            return True
        return False

    def _alloc(self, ns: _NodeSet, slot: int) -> Dict[str, List[int]]:
        """Device ids of slot ``slot`` of a set (g GPUs per slot)."""
        g = ns.g
        if g >= self.gpn:
            return {n: list(range(self.gpn)) for n in ns.nodes}
        base = slot * g
        node = ns.nodes[min(base // self.gpn, len(ns.nodes) - 1)]
        return {node: list(range(base % self.gpn, base % self.gpn + g))}

    # ------------------------------------------------------------ adjust
    def _adjust(self) -> None:
        demand = {g: len([j for ns in lst for j in ns.jobs]) * g for g, lst in self.sets.items()}
        total = sum(demand.values())
        if total == 0:
            return
        for g, lst in self.sets.items():
            if demand[g] == 0:
                continue
            occupied = sum(len(ns.nodes) for ns in lst) * self.gpn
            plan = int(math.floor(demand[g] / total * self.num_gpus))
            target = min(plan, demand[g])
            diff = target - occupied
            if diff > 0:
                self._expand(g, int(math.ceil(diff / g)))
            elif diff < 0:
                self._shrink(g, int(math.ceil(-diff / g)))

    def _respread(self, g: int, jobs: List[Job]) -> None:
        for j in jobs:
            lst = self._sorted(g)
            lst[0].jobs.append(j)

    def _expand(self, g: int, n: int) -> None:
        added = 0
        for _ in range(n):
            if self._new_set(g) is None:
                break
            added += 1
        if added:
            jobs = [j for ns in self.sets[g] for j in ns.jobs]
            for ns in self.sets[g]:
                ns.jobs = []
            self._respread(g, jobs)

    def _shrink(self, g: int, n: int) -> None:
        lst = self._sorted(g)
        n = min(n, len(lst) - 1)                  # never dissolve the last set of a class
        moved: List[Job] = []
        for _ in range(max(0, n)):
            ns = lst.pop(0)
            moved.extend(ns.jobs)
            self.free.extend(ns.nodes)
        if moved:
            self._respread(g, moved)

    # ------------------------------------------------------------ execution
    def _running_view(self) -> Dict[str, tuple]:
        run = {}
        for lst in self.sets.values():
            for ns in lst:
                acc = 0.0
                for slot, j in enumerate(ns.jobs):
                    acc += self._mu(j)
                    if acc > ns.capacity + 1e-9:
                        break
                    run[j.job_id] = (ns, slot)
        return run

    def _sync_states(self) -> int:
        """Bring Job states in line with the node-set view; returns busy GPUs."""
        run = self._running_view()
        busy = 0
        for lst in self.sets.values():
            for ns in lst:
                for j in ns.jobs:
                    if j.job_id in run:
                        if j.state == JobState.PENDING:
                            j.start(self.now, self._alloc(ns, run[j.job_id][1]))
                            self.log.decision(self.now, "start", j.job_id)
                        busy += j.num_gpu
                    elif j.state == JobState.RUNNING:
                        j.preempt(self.now)
                        self.log.decision(self.now, "slice-out", j.job_id)
        return min(busy, self.num_gpus)

    def _execute(self, t1: float) -> bool:
        """Advance running jobs to t1, finishing those that complete; True if
        a node set was released."""
        released = False
        for g, lst in self.sets.items():
            for ns in list(lst):
                for j in list(ns.jobs):
                    if j.state != JobState.RUNNING:
                        continue
                    t_end = self.now + j.time_to_finish()
                    if t_end <= t1 + 1e-9:
                        j.advance(min(t_end, t1))
                        j.progress = j.spec.duration
                        j.finish(min(t_end, t1))
                        ns.jobs.remove(j)
                        self.log.job_row(j.end_time, j)
                        self.log.decision(j.end_time, "finish", j.job_id)
                    else:
                        j.advance(t1)
                if not ns.jobs:
                    lst.remove(ns)
                    self.free.extend(ns.nodes)
                    released = True
        for j in self.pending:
            j.advance(t1)
        for lst in self.sets.values():
            for ns in lst:
                for j in ns.jobs:
                    if j.state == JobState.PENDING:
                        j.advance(t1)
        return released

    def _rotate(self) -> None:
        run = self._running_view()
        for lst in self.sets.values():
            for ns in lst:
                conc = sum(1 for j in ns.jobs if j.job_id in run)
                if len(ns.jobs) > conc:
                    ns.jobs = ns.jobs[conc:] + ns.jobs[:conc]

    # ------------------------------------------------------------ loop
    def run(self, max_ticks: int = 50_000_000) -> Dict:
        t0 = time.perf_counter()
        ai = 0
        self.now = self.arrivals[0].submit_time if self.arrivals else 0.0
        for _ in range(max_ticks):
            self._adjust()
            # arrivals at now
            while ai < len(self.arrivals) and self.arrivals[ai].submit_time <= self.now + 1e-9:
                j = Job(spec=self.arrivals[ai])
                j.arrive(self.now)
                self.jobs[j.job_id] = j
                if self._nodes_for(_pow2_class(j.num_gpu)) > self.total_nodes:
                    j.state = JobState.FAILED               # can never fit this cluster
                    self.log.decision(self.now, "failed", j.job_id)
                elif not self._place(j):
                    self.pending.append(j)
                ai += 1
            busy = self._sync_states()
            if not self.pending and ai >= len(self.arrivals) and \
                    not any(ns.jobs for lst in self.sets.values() for ns in lst):
                break
            nxt = self.now + self.tick
            if ai < len(self.arrivals):
                nxt = min(nxt, self.arrivals[ai].submit_time)
            self.log.account(self.now, busy)
            released = self._execute(nxt)
            self.now = nxt
            if abs(self.now / self.slice - round(self.now / self.slice)) < 1e-9:
                self._rotate()
            if (released or self.free) and self.pending:
                still = []
                for j in self.pending:
                    if not self._place(j):
                        still.append(j)
                self.pending = still
            n_run = sum(1 for j in self.jobs.values() if j.is_running)
            used = sum(j.num_gpu for j in self.jobs.values() if j.is_running)
            self.log.gandiva_row(self.now, len(self.free), min(used, self.num_gpus),
                                 self.num_gpus - min(used, self.num_gpus) - len(self.free) * self.gpn,
                                 len(self.pending), n_run, {g: len(v) for g, v in self.sets.items()})
        else:
            raise RuntimeError("gandiva-ns: tick budget exhausted")
        self.log.account(self.now, 0)
        self.wall_s = time.perf_counter() - t0
        return self.summary()

    def summary(self) -> Dict:
        return self.log.summary(list(self.jobs.values()), self.num_gpus, self.wall_s,
                                extra=dict(schedule="gandiva-ns", scheme="node-set",
                                           mem_util=self.mem_mode))
