"""Placement engine: given a job and the cluster state, return a *plan*
(per task: node + devices) or ``None``; never mutates the cluster (the engine
commits the plan atomically, see ``cluster/topology.py``).

Schemes (reference flag help ``run_sim.py:26-36`` + live ``algorithm.py:
182-187``):

=========  ==============================================================
count      resource counting: any free GPUs, node order (legacy "count")
yarn       consolidated: one node if the gang fits (first-fit, reference
           ``try_single_node_alloc_ms``), else fewest nodes within one rack
           if possible, fullest-free nodes first (``try_cross_node_alloc_ms``)
random     every task on a random node with room (seeded)
crandom    consolidate if one node fits, else random
greedy     nodes with the most free GPUs first
balance    each task to the node with the most free GPUs at that moment
cbalance   consolidate if one node fits, else balance
horus      score-based co-location (reference ``algorithm.py:34-180`` +
horus+     ``horus.py:25-49``): per-device cost = 1.3*mem + util/100 +
gandiva    #tasks, candidate nodes by min cost, fill from racks by
           distance, keep the plan with the fewest nodes
pack       GPU sharing by memory, best fit (legacy ``dlas-gpu-pack``)
tiresias   skew-aware: placement-sensitive models (high largest-tensor /
           total ratio) are consolidated or wait; insensitive ones take
           fragments (best-fit on the fullest nodes, keeping whole nodes
           free for sensitive gangs)
lp         MILP (scipy HiGHS): minimise #nodes (inter-node traffic) then
           fragmentation; the reference's CPLEX LP (``core/lp.py``) is a stub
=========  ==============================================================
"""
from __future__ import annotations

import math
import random
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from ..cluster.topology import Cluster, Node, Plan
from ..core.job import Job, Task

UTILCOST = 1.6    # reference horus.py:1
MEMCOST = 1.3     # reference horus.py:2


class _Scratch:
    """Tentative free-resource view used while building a plan."""

    def __init__(self, cluster: Cluster):
        self.cluster = cluster
        self.cpu = {nid: n.cpu_free() for nid, n in cluster.nodes.items()}
        self.mem = {nid: n.mem_free() for nid, n in cluster.nodes.items()}
        self.dev_tasks = {(nid, d.device_id): len(d.tasks) for nid, n in cluster.nodes.items()
                          for d in n.devices}
        self.dev_mem = {(nid, d.device_id): d.memory_used() for nid, n in cluster.nodes.items()
                        for d in n.devices}
        self.dev_util = {(nid, d.device_id): d.utilization() for nid, n in cluster.nodes.items()
                         for d in n.devices}

    def free_devs(self, nid: str) -> List[int]:
        n = self.cluster.nodes[nid]
        return [d.device_id for d in n.devices if self.dev_tasks[(nid, d.device_id)] == 0]

    def n_free(self, nid: str) -> int:
        return len(self.free_devs(nid))

    def host_ok(self, nid: str, t: Task) -> bool:
        return self.cpu[nid] >= t.cpu and self.mem[nid] >= t.mem

    def dev_ok(self, nid: str, d: int, t: Task, pack: bool) -> bool:
        c = self.cluster
        k = (nid, d)
        if self.dev_tasks[k] > 0 and not pack:
            return False
        if self.dev_tasks[k] >= (c.max_tasks if pack else 1):
            return False
        if pack:
            mem = c.nodes[nid].devices[d].memory
            return mem - (self.dev_mem[k] + t.gpu_mem_max) > c.headroom
        return True

    def take(self, nid: str, devs: Sequence[int], t: Task) -> None:
        self.cpu[nid] -= t.cpu
        self.mem[nid] -= t.mem
        for d in devs:
            self.dev_tasks[(nid, d)] += 1
            self.dev_mem[(nid, d)] += t.gpu_mem_max
            self.dev_util[(nid, d)] = min(100.0, self.dev_util[(nid, d)] + t.gpu_util_avg)

    def try_task(self, nid: str, t: Task, pack: bool = False,
                 dev_key: Optional[Callable[[str, int], float]] = None) -> Optional[Tuple[int, ...]]:
        if not self.host_ok(nid, t):
            return None
        n = self.cluster.nodes[nid]
        cands = [d.device_id for d in n.devices if self.dev_ok(nid, d.device_id, t, pack)]
        if dev_key is not None:
            cands.sort(key=lambda d: dev_key(nid, d))
        if len(cands) < t.gpu:
            return None
        devs = tuple(cands[:t.gpu])
        self.take(nid, devs, t)
        return devs


def _fill(cluster: Cluster, job: Job, node_order: Sequence[str], pack: bool = False,
          scratch: Optional[_Scratch] = None) -> Optional[Plan]:
    s = scratch or _Scratch(cluster)
    plan: Plan = []
    for t in job.tasks:
        for nid in node_order:
            devs = s.try_task(nid, t, pack)
            if devs is not None:
                plan.append((nid, devs))
                break
        else:
            return None
    return plan


def _single_node(cluster: Cluster, job: Job, node_order: Sequence[str]) -> Optional[Plan]:
    for nid in node_order:
        p = _fill(cluster, job, [nid])
        if p is not None:
            return p
    return None


class Placement:
    name = "base"

    def __init__(self, cluster_gpus_per_node: int = 8, rng: Optional[random.Random] = None,
                 sensitivity: Optional[Callable[[Job], bool]] = None, pack: bool = False):
        self.gpn = cluster_gpus_per_node
        self.rng = rng or random.Random(0)
        self.sensitivity = sensitivity
        self.pack = pack
        # set by the engine when GPU sharing is on: model of a placed job and
        # the measured co-run slowdown of a model pair (cluster/interference.py)
        self.model_of: Optional[Callable[[str], str]] = None
        self.pair_cost: Optional[Callable[[str, str], float]] = None
        self.share_max_slowdown = float("inf")
        # set by the engine (engine/spread.py): wait-vs-spread advice for
        # insensitive gangs, and the engine's job table it consults
        self.advisor = None
        self.jobs_by_id: Optional[Dict[str, Job]] = None
        # with the advisor: may a gang that fits one node be fragmented?
        # (spread_rule "wait": yes, when the rule says so; "node": never)
        self.spread_node_gangs = True
        # TiresiasPlacement: decisions per sensitivity verdict, and "flips":
        # placements the other verdict would have planned differently
        self.oracle_stats = {"sensitive": 0, "insensitive": 0, "flips": 0, "flips_sensitive": 0,
                             "flips_insensitive": 0}

    def plan(self, cluster: Cluster, job: Job) -> Optional[Plan]:
        raise NotImplementedError


class CountPlacement(Placement):
    name = "count"

    def plan(self, cluster, job):
        return _fill(cluster, job, list(cluster.nodes))


class YarnPlacement(Placement):
    """Consolidated (YARN-CS / Tiresias default)."""
    name = "yarn"

    def plan(self, cluster, job):
        gpn = max(n.gpu_count for n in cluster.nodes.values())
        order = list(cluster.nodes)
        if job.num_gpu <= gpn:
            p = _single_node(cluster, job, order)
            if p is not None:
                return p
            return None   # a gang that fits a node must not be split (reference semantics)
        # cross-node: prefer a single rack, fullest-free nodes first
        for rid in cluster.racks:
            nodes = sorted(cluster.racks[rid].nodes, key=lambda nid: -cluster.nodes[nid].num_free_gpus())
            if sum(cluster.nodes[n].num_free_gpus() for n in nodes) >= job.num_gpu:
                p = _fill(cluster, job, nodes)
                if p is not None:
                    return p
        nodes = sorted(order, key=lambda nid: -cluster.nodes[nid].num_free_gpus())
        return _fill(cluster, job, nodes)


class RandomPlacement(Placement):
    name = "random"

    def plan(self, cluster, job):
        s = _Scratch(cluster)
        plan: Plan = []
        ids = list(cluster.nodes)
        for t in job.tasks:
            cand = [nid for nid in ids if s.host_ok(nid, t) and s.n_free(nid) >= t.gpu]
            if not cand:
                return None
            nid = self.rng.choice(cand)
            devs = s.try_task(nid, t)
            plan.append((nid, devs))
        return plan


class CRandomPlacement(RandomPlacement):
    name = "crandom"

    def plan(self, cluster, job):
        fits = [nid for nid, n in cluster.nodes.items() if n.num_free_gpus() >= job.num_gpu]
        self.rng.shuffle(fits)
        p = _single_node(cluster, job, fits)
        return p if p is not None else super().plan(cluster, job)


class GreedyPlacement(Placement):
    name = "greedy"

    def plan(self, cluster, job):
        order = sorted(cluster.nodes, key=lambda nid: (-cluster.nodes[nid].num_free_gpus(), int(nid)))
        return _fill(cluster, job, order)


class BalancePlacement(Placement):
    name = "balance"

    def plan(self, cluster, job):
        s = _Scratch(cluster)
        plan: Plan = []
        for t in job.tasks:
            order = sorted(cluster.nodes, key=lambda nid: (-s.n_free(nid), int(nid)))
            for nid in order:
                devs = s.try_task(nid, t)
                if devs is not None:
                    plan.append((nid, devs))
                    break
            else:
                return None
        return plan


class CBalancePlacement(BalancePlacement):
    name = "cbalance"

    def plan(self, cluster, job):
        p = _single_node(cluster, job, list(cluster.nodes))
        return p if p is not None else super().plan(cluster, job)


def horus_cost(util: float, mem_used: float, mem_cap: float, ntasks: int, t: Task,
               gandiva: bool = False) -> float:
    """Per-device cost (reference horus.py:4-49, with the mem-cost precedence
    fixed: (current + task) / capacity)."""
    mem_cost = (mem_used + t.gpu_mem_max) / mem_cap
    if gandiva:
        util_cost = util
    else:
        util_cost = util + t.gpu_util_max - 100.0
        util_cost = util_cost * UTILCOST if util_cost > 0 else abs(util_cost)
    return mem_cost * MEMCOST + util_cost / 100.0 + ntasks


class HorusPlacement(Placement):
    name = "horus"
    gandiva = False

    def plan(self, cluster, job):
        s0 = _Scratch(cluster)
        t0 = job.tasks[0]

        def dev_cost(s: _Scratch, nid: str, d: int) -> float:
            k = (nid, d)
            return horus_cost(s.dev_util[k], s.dev_mem[k], cluster.nodes[nid].devices[d].memory,
                              s.dev_tasks[k], t0, self.gandiva)

        scored = []
        for n in cluster.free_nodes():
            costs = [dev_cost(s0, n.node_id, d.device_id) for d in n.devices
                     if s0.dev_ok(n.node_id, d.device_id, t0, True)]
            if costs and s0.host_ok(n.node_id, t0):
                scored.append((min(costs), int(n.node_id), n.node_id))
        scored.sort()
        cands = scored[:max(1, job.num_gpu)]
        best: Optional[Plan] = None
        best_nodes = None
        for _, _, cnid in cands:
            s = _Scratch(cluster)
            key = (lambda nid, d, s=s: dev_cost(s, nid, d))
            plan: Plan = []
            ok = True
            for t in job.tasks:
                devs = s.try_task(cnid, t, True, key)
                if devs is not None:
                    plan.append((cnid, devs))
                    continue
                placed = False
                for rid in cluster.racks_by_distance(cluster.nodes[cnid].rack_id):
                    for nid in cluster.racks[rid].nodes:
                        devs = s.try_task(nid, t, True, key)
                        if devs is not None:
                            plan.append((nid, devs))
                            placed = True
                            break
                    if placed:
                        break
                if not placed:
                    ok = False
                    break
            if ok:
                nn = len({nid for nid, _ in plan})
                if best is None or nn < best_nodes:
                    best, best_nodes = plan, nn
        return best


class GandivaPlacement(HorusPlacement):
    name = "gandiva"
    gandiva = True


class PackPlacement(Placement):
    """GPU sharing by memory: best-fit the fullest device that still has room."""
    name = "pack"

    def plan(self, cluster, job):
        s = _Scratch(cluster)
        plan: Plan = []
        for t in job.tasks:
            best = None
            for nid, n in cluster.nodes.items():
                if not s.host_ok(nid, t):
                    continue
                devs = [d.device_id for d in n.devices if s.dev_ok(nid, d.device_id, t, True)]
                if len(devs) < t.gpu:
                    continue
                devs.sort(key=lambda d: -s.dev_mem[(nid, d)])
                score = sum(s.dev_mem[(nid, d)] for d in devs[:t.gpu])
                if best is None or score > best[0]:
                    best = (score, nid, tuple(devs[:t.gpu]))
            if best is None:
                return None
            _, nid, devs = best
            s.take(nid, devs, t)
            plan.append((nid, devs))
        return plan


class TiresiasPlacement(Placement):
    """Skew-aware consolidation (Tiresias NSDI'19 §4.3): only jobs whose model
    is placement-sensitive insist on a consolidated gang."""
    name = "tiresias"

    def plan(self, cluster, job):
        p = self._exclusive(cluster, job)
        if p is not None or not (self.pack and cluster.pack) or job.num_gpu != 1:
            return p
        return self._share(cluster, job)

    def _share(self, cluster, job) -> Optional[Plan]:
        """Work-conserving GPU sharing (the reference's --pack / Gandiva
        packing), used only when no GPU is free: a 1-GPU job
        joins a device that holds only 1-GPU jobs and has memory for it,
        choosing the partner with the best measured co-run throughput
        (lowest pair slowdown, profiles/stream_sharing_mi355x.json). The
        executor runs co-located jobs on separate HIP streams. Gangs never
        share, so no rank interleaves two jobs' collectives."""
        t = job.tasks[0]
        s = _Scratch(cluster)
        me = job.spec.model or ""
        best = None
        for nid, n in cluster.nodes.items():
            if not s.host_ok(nid, t):
                continue
            for d in n.devices:
                if not d.tasks or not s.dev_ok(nid, d.device_id, t, True):
                    continue
                occ = [x.job_id for x in d.tasks.values()]
                if any(sum(len(dv) for _, dv in cluster.placed.get(o, [("", (0, 0))])) != 1 for o in occ):
                    continue
                cost, ok = 0.0, True
                for o in occ:
                    other = self.model_of(o) if self.model_of else ""
                    c = max(self.pair_cost(me, other), self.pair_cost(other, me)) if self.pair_cost else 1.0
                    # optional cut-off for bad pairs (for two jobs alone, co-running
                    # at slowdown s beats LAS's run-the-short-one-first iff s < 1.5;
                    # with queues behind them sharing every measured pair won on
                    # 12 seeded traces, so the default admits all)
                    ok = ok and c < self.share_max_slowdown
                    cost += c
                if not ok:
                    continue
                key = (len(occ), cost, int(nid), d.device_id)
                if best is None or key < best[0]:
                    best = (key, nid, d.device_id)
        if best is None:
            return None
        _, nid, dev = best
        return [(nid, (dev,))]

    def _exclusive(self, cluster, job):
        gpn = max(n.gpu_count for n in cluster.nodes.values())
        sensitive = bool(self.sensitivity and self.sensitivity(job))
        min_nodes = max(1, math.ceil(job.num_gpu / gpn))
        if sensitive:
            p = self._consolidated(cluster, job, gpn)
        else:
            p = self._insensitive(cluster, job, gpn, min_nodes, count=True)
        if self.sensitivity is not None:
            # the skew oracle's effect, counted: would the OTHER verdict have
            # placed this job differently right now (another node set, or
            # start vs wait)? Plans are side-effect free; the counterfactual
            # does not touch the advisor's decision counts
            alt = (self._insensitive(cluster, job, gpn, min_nodes, count=False) if sensitive
                   else self._consolidated(cluster, job, gpn))
            st = self.oracle_stats
            st["sensitive" if sensitive else "insensitive"] += 1
            if _plan_key(alt) != _plan_key(p):
                st["flips"] += 1
                st["flips_" + ("sensitive" if sensitive else "insensitive")] += 1
        return p

    def _consolidated(self, cluster, job, gpn):
        """A placement-sensitive job: best-fit single node, or exactly
        min_nodes whole nodes (one rack first), else wait."""
        if job.num_gpu <= gpn:
            order = sorted(cluster.nodes, key=lambda nid: (cluster.nodes[nid].num_free_gpus(), int(nid)))
            return _single_node(cluster, job, order)
        whole = [nid for nid, n in cluster.nodes.items() if n.num_free_gpus() == n.gpu_count]
        if len(whole) * gpn >= job.num_gpu:
            # prefer whole nodes within one rack
            by_rack: Dict[str, List[str]] = {}
            for nid in whole:
                by_rack.setdefault(cluster.nodes[nid].rack_id, []).append(nid)
            for rid, nodes in sorted(by_rack.items(), key=lambda kv: -len(kv[1])):
                if len(nodes) * gpn >= job.num_gpu:
                    return _fill(cluster, job, nodes)
            return _fill(cluster, job, whole)
        return None

    def _insensitive(self, cluster, job, gpn, min_nodes, count: bool):
        # insensitive: fill fragments first (fewest free GPUs first), keep whole nodes
        order = sorted(cluster.nodes, key=lambda nid: (cluster.nodes[nid].num_free_gpus() == 0,
                                                      cluster.nodes[nid].num_free_gpus(), int(nid)))
        if self.advisor is None:
            return _fill(cluster, job, order)
        # with wait-vs-spread advice (engine/spread.py): a gang that fits one
        # node takes the best-fit node when one is free (no link time at
        # all); otherwise the fragments, but only when the expected wait for
        # a consolidated block exceeds what spreading costs it
        if job.num_gpu <= gpn:
            best = sorted(cluster.nodes, key=lambda nid: (cluster.nodes[nid].num_free_gpus(), int(nid)))
            p = _single_node(cluster, job, best)
            if p is not None:
                return p
            if not self.spread_node_gangs:
                # spread_rule "node": a gang that fits one node waits for one
                # (spreading it trades a short wait for a slower rate over its
                # whole run AND fragments the nodes the gangs queued behind it
                # need; priced 10k sweep, profiles/r5/spread_node_rule.md)
                return None
        elif not self.spread_node_gangs:
            # ... and a gang wider than a node packs the fullest-free nodes
            # first (fewest nodes, no fragment of a busy node unless needed)
            order = sorted(cluster.nodes, key=lambda nid: (-cluster.nodes[nid].num_free_gpus(), int(nid)))
        p = _fill(cluster, job, order)
        if p is None:
            return None
        k = len({nid for nid, _ in p})
        if k <= min_nodes or self.advisor.should_spread(cluster, job, self.jobs_by_id or {}, k, gpn, min_nodes,
                                                        count=count):
            return p
        return None


def _plan_key(p):
    return None if p is None else tuple(sorted((nid, tuple(sorted(d))) for nid, d in p))


def _next_pow2(n: int) -> int:
    b = 1
    while b < n:
        b *= 2
    return b


def buddy_pick(free: Sequence[bool], count: int) -> Optional[Tuple[int, ...]]:
    """Best-fit buddy choice on one node: the first ``count`` devices of a
    fully free ALIGNED block of size next_pow2(count), choosing the block
    whose enclosing free aligned region is smallest (fill a half-used pair
    before breaking a free quad), lowest offset on ties. None if no aligned
    block is free."""
    n = len(free)
    b = _next_pow2(max(1, count))
    if b > n:
        return None
    best = None
    for lo in range(0, n - b + 1, b):
        if not all(free[lo:lo + b]):
            continue
        size = b
        while size * 2 <= n:
            plo = lo // (size * 2) * (size * 2)
            if plo + 2 * size <= n and all(free[plo:plo + 2 * size]):
                size *= 2
            else:
                break
        key = (size, lo)
        if best is None or key < best:
            best = key
    return None if best is None else tuple(range(best[1], best[1] + count))


def align_plan(cluster: Cluster, job: Job, plan: Optional[Plan]) -> Optional[Plan]:
    """Canonical gang rank sets (``--gang_align``, on for the live MI355X
    runtime). Keeps the placement's choice of NODES but moves each node's
    share of the gang onto an aligned buddy block of devices, so every
    power-of-two gang runs on one of the ``2*gpn - 1 - gpn`` canonical rank
    sets (``parallel/gang.py::canonical_gang_sets``) whose RCCL
    communicators are created once, outside the timed region, instead of
    one communicator per arbitrary device subset (up to 247 on 8 GPUs).
    1-GPU jobs are best-fit too, which is what keeps aligned blocks free.
    Shared (packed) placements are left alone. When the chosen node has
    enough free GPUs but no aligned block, a single-node gang moves to the
    best-fitting node that has one; otherwise the job waits (None)."""
    if plan is None:
        return None
    for nid, devs in plan:
        node = cluster.nodes[nid]
        if any(node.devices[d].tasks for d in devs):
            return plan                                # GPU sharing: not a gang rank set
    per_node: Dict[str, int] = {}
    for nid, devs in plan:
        per_node[nid] = per_node.get(nid, 0) + len(devs)

    def free_of(nid):
        return [not d.tasks for d in cluster.nodes[nid].devices]

    blocks = {nid: buddy_pick(free_of(nid), c) for nid, c in per_node.items()}
    if any(b is None for b in blocks.values()):
        if len(per_node) != 1:
            return None
        c = job.num_gpu
        s = _Scratch(cluster)
        best = None
        for nid in cluster.nodes:
            if not all(s.host_ok(nid, t) for t in job.tasks):
                continue
            fr = free_of(nid)
            blk = buddy_pick(fr, c)
            if blk is not None:
                key = (sum(fr), int(nid))                # fullest node first (best fit)
                if best is None or key < best[0]:
                    best = (key, nid, blk)
        if best is None:
            return None
        _, nid, blk = best
        blocks = {nid: blk}
        plan = [(nid, devs) for _, devs in plan]
    out: Plan = []
    used = {nid: 0 for nid in blocks}
    for nid, devs in plan:
        k = used[nid]
        out.append((nid, tuple(blocks[nid][k:k + len(devs)])))
        used[nid] = k + len(devs)
    return out


PLACEMENTS = {c.name: c for c in (CountPlacement, YarnPlacement, RandomPlacement, CRandomPlacement,
                                  GreedyPlacement, BalancePlacement, CBalancePlacement, HorusPlacement,
                                  GandivaPlacement, PackPlacement, TiresiasPlacement)}
PLACEMENTS["horus+"] = HorusPlacement


def make_placement(name: str, **kw) -> Placement:
    if name == "lp":
        from .lp import LPPlacement

        return LPPlacement(**kw)
    if name not in PLACEMENTS:
        raise ValueError(f"unknown placement scheme {name!r}; choose from {sorted(PLACEMENTS) + ['lp']}")
    return PLACEMENTS[name](**kw)
