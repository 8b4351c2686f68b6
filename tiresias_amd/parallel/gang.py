"""Gang communicators: how a DDP gang's gradient all-reduce travels.

Tiresias' placement problem exists because a gang spread over several nodes
pays the slow inter-node network for every all-reduce, while a consolidated
gang stays on the fast intra-node fabric (reference: the rack/node hierarchy
``infra/infrastructure.py:45-69`` and the cost model
``core/network/network_service.py:3-39``). One MI355X node is a fully
connected xGMI mesh, so the cluster runtime partitions it into VIRTUAL nodes
(``--virtual_nodes 2x4``) and gives gangs that cross a virtual-node boundary a
real inter-node transport instead of the free xGMI path:

* ``FlatComm`` (consolidated gang): one RCCL communicator over xGMI, bucketed
  in-place ``all_reduce`` (RCCL's multi-channel rings use every link).
* ``HierComm`` (spread gang), per gradient bucket, three phases:
    1. intra-virtual-node RCCL ``reduce`` to the part's leader (xGMI);
    2. leaders exchange through PINNED HOST buffers on a side stream — D2H,
       a gloo all-reduce among the leaders (the "NIC"), H2D — throttled to
       ``nic_gbps`` per leader (a calibrated NIC rate, default 12.5 GB/s =
       100 Gb/s) plus a per-message latency, on a leader-side worker thread
       so backward keeps issuing kernels while buckets are in flight;
    3. intra-virtual-node RCCL ``broadcast`` from the leader.
  The compute stream waits on an event, never the host, except in
  ``finish`` (end of backward) where the host joins the exchange thread.

The same factory builds the communicators for the training runtime
(``executor/cluster_runtime.py``) and the skew profiler
(``profiler/comm.py``), so what the profiler measures is what jobs pay.
``create_gang_comm`` builds member-only communicators (``GangPG``): only the
gang's members rendezvous, so gangs form and dissolve freely and a lost rank
elsewhere does not block anything.
"""
from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import Future
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

DEFAULT_NIC_GBPS = 12.5          # 100 Gb/s: the emulated inter-node link per GPU
DEFAULT_NIC_LATENCY_S = 10e-6


def vnode_parts(ranks: Sequence[int], vnode_size: int) -> List[List[int]]:
    """Split a gang's ranks by virtual node (rank // vnode_size), in order."""
    ranks = sorted(int(r) for r in ranks)
    if vnode_size <= 0:
        return [ranks]
    parts: Dict[int, List[int]] = {}
    for r in ranks:
        parts.setdefault(r // vnode_size, []).append(r)
    return [parts[k] for k in sorted(parts)]


def ring_exchange_bytes(nbytes: float, k: int) -> float:
    """Bytes each of k participants sends in a ring all-reduce of nbytes."""
    return 0.0 if k <= 1 else 2.0 * (k - 1) / k * nbytes


class FlatComm:
    kind = "flat"

    def __init__(self, pg, ranks: Sequence[int]):
        self.pg = pg
        self.ranks = tuple(ranks)
        self.size = len(self.ranks)

    def start(self, view: torch.Tensor):
        return self.pg.all_reduce(view)

    def finish(self, handles) -> None:
        for w in handles:
            w.wait()

    def close(self) -> None:
        pass


class _NicLimiter:
    """Enforces a per-leader NIC rate: an exchange of ``b`` bytes takes at
    least latency + b / rate."""

    def __init__(self, gbps: float, latency_s: float):
        self.rate = gbps * 1e9
        self.latency = latency_s
        self.bytes = 0.0
        self.busy_s = 0.0

    def throttle(self, sent_bytes: float, t0: float) -> None:
        need = self.latency + (sent_bytes / self.rate if self.rate > 0 else 0.0)
        left = need - (time.perf_counter() - t0)
        if left > 0:
            time.sleep(left)
        self.bytes += sent_bytes
        self.busy_s += max(need, time.perf_counter() - t0)


class HierComm:
    kind = "hier"

    def __init__(self, ranks: Sequence[int], parts: List[List[int]], my_rank: int, local_pgs: Dict[int, object],
                 leaders_pg, device: torch.device, nic_gbps: float = DEFAULT_NIC_GBPS,
                 nic_latency_s: float = DEFAULT_NIC_LATENCY_S):
        self.ranks = tuple(ranks)
        self.size = len(self.ranks)
        self.parts = parts
        self.device = device
        mine = next(p for p in parts if my_rank in p)
        self.part = mine
        self.leader = mine[0]
        self.is_leader = my_rank == self.leader
        self.local_pg = local_pgs.get(mine[0])          # None when the part is a single rank
        self.leaders_pg = leaders_pg
        self.k = len(parts)
        self.nic = _NicLimiter(nic_gbps, nic_latency_s)
        self._cuda = device.type == "cuda"
        self._side = torch.cuda.Stream(device) if (self._cuda and self.is_leader) else None
        self._host: Dict[int, torch.Tensor] = {}
        self._q: Optional[queue.Queue] = None
        self._th: Optional[threading.Thread] = None
        if self.is_leader:
            self._q = queue.Queue()
            self._th = threading.Thread(target=self._loop, name=f"nic-{my_rank}", daemon=True)
            self._th.start()

    # --------------------------------------------------------------- leader thread
    def _pinned(self, n: int) -> torch.Tensor:
        t = self._host.get(n)
        if t is None:
            t = torch.empty(n, dtype=torch.float32, pin_memory=True)
            self._host[n] = t
        return t

    def _loop(self) -> None:
        if self._cuda:
            torch.cuda.set_device(self.device)
        while True:
            item = self._q.get()
            if item is None:
                return
            view, work, fut = item
            try:
                fut.set_result(self._exchange(view, work))
            except BaseException as e:          # surfaced in finish()
                fut.set_exception(e)

    def _exchange(self, view: torch.Tensor, work):
        nbytes = view.numel() * view.element_size()
        if self._cuda:
            with torch.cuda.stream(self._side):
                if work is not None:
                    work.wait()                  # side stream after the intra-node reduce
                host = self._pinned(view.numel())
                host.copy_(view, non_blocking=True)
                self._side.synchronize()         # D2H landed (this thread only)
        else:
            if work is not None:
                work.wait()
            host = view
        t0 = time.perf_counter()
        self.leaders_pg.all_reduce(host).wait()
        self.nic.throttle(ring_exchange_bytes(nbytes, self.k), t0)
        if not self._cuda:
            return None
        with torch.cuda.stream(self._side):
            view.copy_(host, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._side)
        return ev

    # --------------------------------------------------------------- bucket API
    def start(self, view: torch.Tensor):
        w = None
        if self.local_pg is not None:
            w = self.local_pg.reduce(view, self.leader)
        fut = None
        if self.is_leader:
            fut = Future()
            self._q.put((view, w, fut))
        return (view, w, fut)

    def finish(self, handles) -> None:
        bcasts = []
        for view, w, fut in handles:
            if fut is not None:
                ev = fut.result()
                if ev is not None:
                    torch.cuda.current_stream(self.device).wait_event(ev)
            elif w is not None:
                w.wait()
            if self.local_pg is not None:
                bcasts.append(self.local_pg.broadcast(view, self.leader))
        for b in bcasts:
            b.wait()

    def close(self) -> None:
        if self._q is not None:
            self._q.put(None)
            self._q = None


_PGS: Dict[tuple, object] = {}
GANG_TIMEOUT_S = float(__import__("os").environ.get("TAM_GANG_TIMEOUT_S", "120"))


class GangPG:
    """A communicator over an arbitrary rank set, built directly on a c10d
    backend (``ProcessGroupNCCL`` = RCCL on ROCm, or ``ProcessGroupGloo``)
    from the job's key-value store under a per-rank-set prefix: only the
    members rendezvous (ncclCommInitRank with a unique id exchanged through
    the store), no world-wide bookkeeping. ``torch.distributed.new_group``
    would need every rank of the world to take part (or, with local
    synchronisation, identical group histories on the members) — neither
    holds once gangs form and dissolve dynamically, or after a rank is lost.
    Collective calls return Work handles (``wait()`` orders the current
    stream after them)."""

    def __init__(self, ranks: Sequence[int], my_rank: int, backend: str, timeout_s: float = GANG_TIMEOUT_S):
        from datetime import timedelta

        self.ranks = tuple(ranks)
        self.rank = self.ranks.index(my_rank)
        self.size = len(self.ranks)
        self.backend = backend
        base = dist.distributed_c10d._get_default_store()
        store = dist.PrefixStore(f"tam/pg/{backend}/{'_'.join(map(str, self.ranks))}", base)
        to = timedelta(seconds=timeout_s)
        if backend == "nccl":
            self.pg = dist.ProcessGroupNCCL(store, self.rank, self.size, to)
        else:
            self.pg = dist.ProcessGroupGloo(store, self.rank, self.size, to)

    def all_reduce(self, t: torch.Tensor):
        o = dist.AllreduceOptions()
        o.reduceOp = dist.ReduceOp.SUM
        return self.pg.allreduce([t], o)

    def reduce(self, t: torch.Tensor, root_global: int):
        o = dist.ReduceOptions()
        o.reduceOp = dist.ReduceOp.SUM
        o.rootRank = self.ranks.index(root_global)
        o.rootTensor = 0
        return self.pg.reduce([t], o)

    def broadcast(self, t: torch.Tensor, root_global: int):
        o = dist.BroadcastOptions()
        o.rootRank = self.ranks.index(root_global)
        o.rootTensor = 0
        return self.pg.broadcast([t], o)


def _pg(ranks: Sequence[int], my_rank: int, backend: str) -> GangPG:
    """One communicator per (rank set, backend) per process (members create
    it the first time they need it; the store prefix is the rank set)."""
    key = (tuple(ranks), backend)
    if key not in _PGS:
        _PGS[key] = GangPG(ranks, my_rank, backend)
    return _PGS[key]


def create_gang_comm(ranks: Sequence[int], my_rank: int, vnode_size: int = 0, backend: str = "nccl",
                     device: Optional[torch.device] = None, nic_gbps: float = DEFAULT_NIC_GBPS,
                     nic_latency_s: float = DEFAULT_NIC_LATENCY_S):
    """Called by every live rank with the same args in the same order (the
    plan broadcast guarantees it); only members rendezvous. Returns this
    rank's comm (None when not a member)."""
    ranks = tuple(sorted(int(r) for r in ranks))
    parts = vnode_parts(ranks, vnode_size)
    device = device or torch.device("cpu")
    if my_rank not in ranks:
        return None
    if len(parts) <= 1:
        return FlatComm(_pg(ranks, my_rank, backend), ranks)
    local_pgs = {}
    for p in parts:
        if len(p) > 1 and my_rank in p:
            local_pgs[p[0]] = _pg(tuple(p), my_rank, backend)
    leaders_pg = None
    leaders = tuple(p[0] for p in parts)
    if my_rank in leaders:
        leaders_pg = _pg(leaders, my_rank, "gloo")
    return HierComm(ranks, parts, my_rank, local_pgs, leaders_pg, device, nic_gbps, nic_latency_s)


def comm_size(group) -> int:
    """World size of a gang comm or a plain process group."""
    if group is None:
        return 1
    if hasattr(group, "size") and not callable(group.size):
        return int(group.size)
    return dist.get_world_size(group)


class _PlainPG:
    """A torch.distributed process group behind the GangPG interface."""

    def __init__(self, pg):
        self.pg = pg

    def all_reduce(self, t):
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)


def as_comm(group):
    """Wrap a plain process group as a FlatComm (legacy callers)."""
    if group is None or isinstance(group, (FlatComm, HierComm)):
        return group
    return FlatComm(_PlainPG(group), tuple(range(dist.get_world_size(group))))
