"""Cluster resource model: racks (switches) x nodes x GPU devices.

Same hierarchy and capacities as the reference (``infra/infrastructure.py:
16-147``, ``infra/rack.py``, ``infra/node.py:7-287``, ``infra/device.py:
4-58``), redesigned around one invariant the reference breaks (defect D2:
``try_reserve_and_placed_task`` mutates counters before knowing a task fits
and never rolls back): **placement is side-effect free**. Placement
algorithms read the cluster and return a *plan*; ``Cluster.commit`` validates
the whole plan and applies it atomically; ``Cluster.release`` returns every
resource. ``check_invariants`` verifies conservation after any event.

MI355X mapping: one 8-GPU node is the real machine; ``virtual_nodes="2x4"``
partitions it into virtual nodes so consolidated-vs-spread placement has a
meaning (spread gangs cross a virtual-node boundary; the executor emulates
the slower path, the simulator charges the network model).
"""
from __future__ import annotations

import random
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from ..config import ClusterSpec
from ..core.job import Job, Task

# plan: per task index -> (node_id, device ids)
Plan = List[Tuple[str, Tuple[int, ...]]]


class Device:
    def __init__(self, device_id: int, node_id: str, memory_mb: float):
        self.device_id = device_id
        self.node_id = node_id
        self.memory = memory_mb
        self.tasks: "OrderedDict[str, Task]" = OrderedDict()
        self.failed = False          # a lost GPU / rank: never placed on again

    def is_idle(self) -> bool:
        return not self.tasks and not self.failed

    def memory_used(self) -> float:
        return min(self.memory, sum(min(self.memory, t.gpu_mem_max) for t in self.tasks.values()))

    def can_fit(self, task: Task, pack: bool, max_tasks: int = 3, headroom_mb: float = 500.0) -> bool:
        if self.failed:
            return False
        if self.tasks and not pack:
            return False
        if len(self.tasks) >= max_tasks:
            return False
        return self.memory - (self.memory_used() + task.gpu_mem_max) > headroom_mb

    def utilization(self, rng: Optional[random.Random] = None) -> float:
        """Expected (rng=None) or sampled utilisation in [0, 100] (defect D9:
        the reference logs an unclamped numpy array)."""
        u = 0.0
        for t in self.tasks.values():
            if rng is None:
                v = t.gpu_util_avg
            else:
                v = rng.gauss(t.gpu_util_avg, max(0.0, (t.gpu_util_max - t.gpu_util_avg) / 2))
            u += min(100.0, max(0.0, v))
        return min(100.0, u)


class Node:
    def __init__(self, node_id: str, rack_id: str, gpus: int, cpus: int, mem: int, gpu_mem_mb: float):
        self.node_id = node_id
        self.rack_id = rack_id
        self.cpu_count = cpus
        self.mem_size = mem
        self.cpu_used = 0
        self.mem_used = 0
        self.devices = [Device(i, node_id, gpu_mem_mb) for i in range(gpus)]
        self.jobs: Dict[str, List[int]] = {}   # job_id -> task indices on this node

    @property
    def gpu_count(self) -> int:
        return len(self.devices)

    def live_gpus(self) -> int:
        return sum(1 for d in self.devices if not d.failed)

    def free_devices(self) -> List[int]:
        return [d.device_id for d in self.devices if d.is_idle()]

    def num_free_gpus(self) -> int:
        return sum(1 for d in self.devices if d.is_idle())

    def cpu_free(self) -> int:
        return self.cpu_count - self.cpu_used

    def mem_free(self) -> int:
        return self.mem_size - self.mem_used

    def is_idle(self) -> bool:
        return not self.jobs

    def can_host(self, task: Task) -> bool:
        return self.cpu_free() >= task.cpu and self.mem_free() >= task.mem


class Rack:
    def __init__(self, rack_id: str, bandwidth: float):
        self.rack_id = rack_id
        self.bandwidth = bandwidth
        self.nodes: "OrderedDict[str, Node]" = OrderedDict()


class PlacementError(RuntimeError):
    pass


class Cluster:
    def __init__(self, spec: ClusterSpec, pack: bool = False, max_tasks_per_gpu: int = 3,
                 headroom_mb: float = 500.0, virtual_nodes: str = ""):
        self.spec = spec
        self.pack = pack
        self.max_tasks = max_tasks_per_gpu
        self.headroom = headroom_mb
        self.racks: "OrderedDict[str, Rack]" = OrderedDict()
        self.nodes: "OrderedDict[str, Node]" = OrderedDict()
        if virtual_nodes:
            # e.g. "2x4": the single physical node is split into 2 virtual nodes of 4 GPUs
            nv, gpv = (int(x) for x in virtual_nodes.lower().split("x"))
            spec = ClusterSpec(**{**spec.__dict__, "num_switch": 1, "num_node_p_switch": nv,
                                  "num_gpu_p_node": gpv})
            self.spec = spec
        nid = 0
        for r in range(spec.num_switch):
            rack = Rack(str(r), spec.bandwidth_mbps)
            for _ in range(spec.num_node_p_switch):
                nid += 1
                n = Node(str(nid), rack.rack_id, spec.num_gpu_p_node, spec.num_cpu_p_node,
                         spec.mem_p_node, spec.gpu_memory_mb)
                rack.nodes[n.node_id] = n
                self.nodes[n.node_id] = n
            self.racks[rack.rack_id] = rack
        self.placed: Dict[str, Plan] = {}

    # ------------------------------------------------------------ queries
    @property
    def num_gpus(self) -> int:
        """Usable GPUs (failed devices excluded)."""
        return sum(n.live_gpus() for n in self.nodes.values())

    def fail_device(self, node_id: str, dev: int) -> None:
        """Take a lost GPU out of the cluster for good. Jobs on it must have
        been released first (the executor preempts them)."""
        d = self.nodes[node_id].devices[dev]
        if d.tasks:
            raise PlacementError(f"device {node_id}:{dev} still hosts {list(d.tasks)}")
        d.failed = True

    def free_gpus(self) -> int:
        return sum(n.num_free_gpus() for n in self.nodes.values())

    def busy_gpus(self) -> int:
        return self.num_gpus - self.free_gpus()

    def free_nodes(self) -> List[Node]:
        """Nodes with any spare CPU or memory (reference ``Node.is_free``)."""
        return [n for n in self.nodes.values() if n.cpu_free() > 0 or n.mem_free() > 0]

    def racks_by_distance(self, rack_id: str) -> List[str]:
        """Racks ordered by |rack_id - r| (reference infrastructure.py:135-147)."""
        ids = list(self.racks)
        base = int(rack_id)
        return sorted(ids, key=lambda r: (abs(int(r) - base), int(r)))

    def device(self, node_id: str, dev: int) -> Device:
        return self.nodes[node_id].devices[dev]

    # ------------------------------------------------------------ commit / release
    def validate(self, job: Job, plan: Plan) -> Optional[str]:
        if len(plan) != len(job.tasks):
            return f"plan covers {len(plan)} of {len(job.tasks)} tasks"
        cpu: Dict[str, int] = {}
        mem: Dict[str, int] = {}
        dev_use: Dict[Tuple[str, int], List[Task]] = {}
        for task, (nid, devs) in zip(job.tasks, plan):
            if nid not in self.nodes:
                return f"unknown node {nid}"
            if len(devs) != task.gpu or len(set(devs)) != len(devs):
                return f"task {task.task_id} needs {task.gpu} distinct devices, got {devs}"
            cpu[nid] = cpu.get(nid, 0) + task.cpu
            mem[nid] = mem.get(nid, 0) + task.mem
            for d in devs:
                if not (0 <= d < self.nodes[nid].gpu_count):
                    return f"bad device {nid}:{d}"
                if self.nodes[nid].devices[d].failed:
                    return f"device {nid}:{d} failed"
                dev_use.setdefault((nid, d), []).append(task)
        for nid, c in cpu.items():
            n = self.nodes[nid]
            if c > n.cpu_free() or mem[nid] > n.mem_free():
                return f"node {nid} lacks cpu/mem"
        for (nid, d), tasks in dev_use.items():
            dv = self.nodes[nid].devices[d]
            if dv.tasks and not self.pack:
                return f"device {nid}:{d} busy"
            if len(dv.tasks) + len(tasks) > (self.max_tasks if self.pack else 1):
                return f"device {nid}:{d} task limit"
            if self.pack:
                need = sum(t.gpu_mem_max for t in tasks)
                if dv.memory - (dv.memory_used() + need) <= self.headroom:
                    return f"device {nid}:{d} out of memory"
        return None

    def commit(self, job: Job, plan: Plan) -> Dict[str, List[int]]:
        err = self.validate(job, plan)
        if err:
            raise PlacementError(f"job {job.job_id}: {err}")
        alloc: Dict[str, List[int]] = {}
        for task, (nid, devs) in zip(job.tasks, plan):
            n = self.nodes[nid]
            n.cpu_used += task.cpu
            n.mem_used += task.mem
            n.jobs.setdefault(job.job_id, []).append(task.index)
            for d in devs:
                n.devices[d].tasks[task.task_id] = task
            task.node_id = nid
            task.devices = tuple(devs)
            alloc.setdefault(nid, []).extend(devs)
        self.placed[job.job_id] = list(plan)
        return alloc

    def release(self, job: Job) -> None:
        plan = self.placed.pop(job.job_id, None)
        if plan is None:
            return
        for task, (nid, devs) in zip(job.tasks, plan):
            n = self.nodes[nid]
            n.cpu_used -= task.cpu
            n.mem_used -= task.mem
            for d in devs:
                n.devices[d].tasks.pop(task.task_id, None)
            task.node_id = None
            task.devices = ()
        for nid in {nid for nid, _ in plan}:
            self.nodes[nid].jobs.pop(job.job_id, None)

    def nodes_of(self, job_id: str) -> List[str]:
        plan = self.placed.get(job_id)
        return sorted({nid for nid, _ in plan}, key=int) if plan else []

    def shared_devices(self, job_id: str) -> bool:
        plan = self.placed.get(job_id) or []
        for nid, devs in plan:
            for d in devs:
                if len(self.nodes[nid].devices[d].tasks) > 1:
                    return True
        return False

    def neighbours(self, job_id: str) -> set:
        """Ids of the other jobs sharing at least one device with ``job_id``."""
        out = set()
        for nid, devs in self.placed.get(job_id) or []:
            for d in devs:
                for t in self.nodes[nid].devices[d].tasks.values():
                    if t.job_id != job_id:
                        out.add(t.job_id)
        return out

    def check_invariants(self) -> None:
        for n in self.nodes.values():
            cpu = mem = 0
            seen = set()
            for dv in n.devices:
                for t in dv.tasks.values():
                    if t.task_id not in seen:
                        seen.add(t.task_id)
                        cpu += t.cpu
                        mem += t.mem
                if len(dv.tasks) > (self.max_tasks if self.pack else 1):
                    raise AssertionError(f"device {n.node_id}:{dv.device_id} over-subscribed")
            if cpu != n.cpu_used or mem != n.mem_used:
                raise AssertionError(f"node {n.node_id}: counters {n.cpu_used}/{n.mem_used} != "
                                     f"tasks {cpu}/{mem} (resource leak)")
            if n.cpu_used < 0 or n.cpu_used > n.cpu_count or n.mem_used > n.mem_size:
                raise AssertionError(f"node {n.node_id}: capacity violated")

    def snapshot(self) -> Dict[str, List[int]]:
        return {nid: n.free_devices() for nid, n in self.nodes.items()}
