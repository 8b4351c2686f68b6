"""Communication / skew profiler: measures the gradient synchronisation a DDP
gang actually performs — the same gang communicators the training runtime
uses (``parallel/gang.py``), driven with each model's real gradient buckets
(``parallel/ddp.py`` bucketing of the model's arena) — on a CONSOLIDATED rank
set (all ranks in one virtual node: one RCCL communicator over xGMI) and a
SPREAD one (crossing the virtual-node boundary: intra-node RCCL + the
host-staged, rate-capped inter-node exchange). The per-model slowdown it
writes is what ``--skew_profile`` feeds to the placement engine's
``SensitivityOracle`` (``profiler/skew.py``), in the simulator and in the
live controller: Tiresias consolidates only the jobs for which spreading
measurably hurts (reference: per-tensor gradient sizes as the skew source,
``core/models.py:8-26``; the network cost ``core/network/network_service.py:
3-39``).

Run on N >= 2 ranks (RCCL on GPUs, gloo on CPU)::

    python -m torch.distributed.run --standalone --nproc-per-node 8 \\
        -m tiresias_amd.profiler.comm --virtual_nodes 2x4 --gang 4 --out profiles/skew.json

Iteration-level slowdown of model m (the number placement uses):
    (t_iter(m) + t_sync_spread(m) - t_sync_consolidated(m)) / t_iter(m)
with t_iter the measured single-GPU step time (the consolidated sync largely
overlaps backward; the spread penalty does not).
"""
from __future__ import annotations

import argparse
import json
import os
import time
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from ..parallel.gang import DEFAULT_NIC_GBPS, create_gang_comm, vnode_parts
from .skew import model_profile
from .step_times import MI355X_STEP_S

# single-GPU hipGraph step seconds on MI355X, this round's kernels
# (profiler/step_times.py); the denominator of the iteration-level slowdown
ITER_S = dict(MI355X_STEP_S)


def ring_busbw(bytes_: float, seconds: float, n: int) -> float:
    """NCCL-convention bus bandwidth of an all-reduce (GB/s)."""
    if seconds <= 0 or n <= 1:
        return 0.0
    return bytes_ * 2 * (n - 1) / n / seconds / 1e9


def model_buckets(model: str, bucket_mb: float = 32.0) -> List[int]:
    """Gradient bucket sizes (fp32 elements) the DDP bucketer cuts for
    ``model`` (reverse registration order, closed at >= bucket_mb)."""
    prof = model_profile(model)
    elems = max(1, int(bucket_mb * (1 << 20) // 4))
    out, cur = [], 0
    for t in reversed(prof.tensors):
        cur += int(t * (1 << 20) / 4)
        if cur >= elems:
            out.append(cur)
            cur = 0
    if cur:
        out.append(cur)
    return out


class CommProfiler:
    def __init__(self, world_group=None, device: Optional[torch.device] = None, iters: int = 10,
                 warmup: int = 3, vnode_size: int = 0, nic_gbps: float = DEFAULT_NIC_GBPS):
        self.world = world_group
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.device = device or (torch.device("cuda", torch.cuda.current_device())
                                 if torch.cuda.is_available() else torch.device("cpu"))
        self.iters = iters
        self.warmup = warmup
        self.vnode_size = vnode_size
        self.nic_gbps = nic_gbps
        self._comms = {}

    def _comm(self, ranks: Sequence[int]):
        key = tuple(sorted(ranks))
        if key not in self._comms:
            backend = "nccl" if self.device.type == "cuda" else "gloo"
            # collective on all ranks
            self._comms[key] = create_gang_comm(key, self.rank, self.vnode_size, backend, self.device,
                                                self.nic_gbps)
        return self._comms[key]

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def _time(self, comm, sizes: List[int]) -> float:
        bufs = [torch.ones(n, dtype=torch.float32, device=self.device) for n in sizes]
        for it in range(self.warmup + self.iters):
            if it == self.warmup:
                self._sync()
                t0 = time.perf_counter()
            comm.finish([comm.start(b) for b in bufs])
        self._sync()
        return (time.perf_counter() - t0) / self.iters

    def time_allreduce(self, ranks: Sequence[int], nbytes: int) -> Optional[float]:
        comm = self._comm(ranks)
        if comm is None:
            return None
        return self._time(comm, [max(1, nbytes // 4)])

    def time_model(self, ranks: Sequence[int], model: str, bucket_mb: float = 32.0) -> Optional[float]:
        """One full gradient synchronisation of ``model`` on ``ranks`` (every
        bucket launched, then joined), seconds."""
        comm = self._comm(ranks)
        if comm is None:
            return None
        return self._time(comm, model_buckets(model, bucket_mb))

    def sweep(self, sizes_mb: Sequence[float], gang_sets: Dict[str, Sequence[int]]) -> Dict:
        """Returns {set_name: {size_mb: seconds}} (valid on member ranks)."""
        out: Dict[str, Dict[float, float]] = {}
        for name, ranks in gang_sets.items():
            self._comm(ranks)
        for name, ranks in gang_sets.items():
            res = {}
            for mb in sizes_mb:
                t = self.time_allreduce(ranks, int(mb * 2 ** 20))
                if t is not None:
                    res[mb] = t
            out[name] = res
            if self.world is not None:
                dist.barrier(group=self.world)
        return out

    def profile_models(self, models: Sequence[str], gang_sets: Dict[str, Sequence[int]],
                       bucket_mb: float = 32.0) -> Dict[str, Dict[str, float]]:
        """{model: {set_name: seconds}} for every model on every gang set
        (times valid on rank 0, which must be a member of every set)."""
        for ranks in gang_sets.values():
            self._comm(ranks)
        out: Dict[str, Dict[str, float]] = {}
        for m in models:
            out[m] = {}
            for name, ranks in gang_sets.items():
                t = self.time_model(ranks, m, bucket_mb)
                if t is not None:
                    out[m][name] = t
                if self.world is not None:
                    dist.barrier(group=self.world)
        return out

    @staticmethod
    def model_time(model: str, per_size: Dict[float, float], bucket_mb: float = 32.0) -> float:
        """Interpolated sync time of a model's buckets from a size sweep."""
        buckets = [n * 4 / 2 ** 20 for n in model_buckets(model, bucket_mb)]
        pts = sorted(per_size.items())
        if not pts:
            return 0.0

        def interp(mb):
            if mb <= pts[0][0]:
                return pts[0][1] * mb / pts[0][0]
            for (a, ta), (b, tb) in zip(pts, pts[1:]):
                if mb <= b:
                    return ta + (tb - ta) * (mb - a) / (b - a)
            a, ta = pts[-1]
            return ta * mb / a

        return sum(interp(b) for b in buckets)

    @staticmethod
    def classify(times: Dict[str, Dict[str, float]], threshold: float = 1.25,
                 iter_s: Optional[Dict[str, float]] = None) -> Dict:
        """Per-model consolidated / spread sync time, iteration-level slowdown
        and the placement-sensitivity verdict (the ``--skew_profile`` JSON)."""
        iter_s = iter_s or ITER_S
        out = {}
        for m, d in times.items():
            tc, ts = d.get("consolidated", 0.0), d.get("spread", 0.0)
            it = iter_s.get(m, 0.01)
            sd = (it + max(0.0, ts - tc)) / it
            out[m] = {"consolidated_s": tc, "spread_s": ts, "sync_ratio": ts / tc if tc > 0 else 1.0,
                      "iter_s": it, "slowdown": sd, "skew": model_profile(m).skew,
                      "sensitive": sd >= threshold}
        return out

    def classify_models(self, models: Sequence[str], sweep: Dict, threshold: float = 1.1) -> Dict:
        """Back-compatible: classify from a size sweep (interpolated)."""
        times = {m: {"consolidated": self.model_time(m, sweep.get("consolidated", {})),
                     "spread": self.model_time(m, sweep.get("spread", {}))} for m in models}
        return self.classify(times, threshold)


def default_gang_sets(world: int, vnode_size: int, gang: int) -> Dict[str, List[int]]:
    """Consolidated = the first ``gang`` ranks of virtual node 0; spread =
    the same number of ranks split evenly over two virtual nodes."""
    cons = list(range(gang))
    half = gang // 2
    spread = list(range(half)) + list(range(vnode_size, vnode_size + gang - half))
    assert len(vnode_parts(cons, vnode_size)) == 1 and len(vnode_parts(spread, vnode_size)) == 2
    assert max(spread) < world
    return {"consolidated": cons, "spread": spread}


def save(path: str, data: Dict) -> None:
    with open(path, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True, default=str)


def main(argv=None) -> Optional[Dict]:
    ap = argparse.ArgumentParser(description="consolidated-vs-spread gradient-sync profiler")
    ap.add_argument("--virtual_nodes", default="2x4")
    ap.add_argument("--gang", type=int, default=4)
    ap.add_argument("--models", default="resnet50,vgg16,transformer,gnmt")
    ap.add_argument("--nic_gbps", type=float, default=DEFAULT_NIC_GBPS)
    ap.add_argument("--threshold", type=float, default=1.25)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--out", default="profiles/skew_profile.json")
    a = ap.parse_args(argv)
    if not dist.is_initialized():
        use_cuda = torch.cuda.is_available()
        if use_cuda:
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
        dist.init_process_group("nccl" if use_cuda else "gloo")
    world = dist.get_world_size()
    nv, gpv = (int(x) for x in a.virtual_nodes.lower().split("x"))
    if nv * gpv != world:
        raise SystemExit(f"--virtual_nodes {a.virtual_nodes} does not cover world {world}")
    prof = CommProfiler(dist.group.WORLD, iters=a.iters, vnode_size=gpv, nic_gbps=a.nic_gbps)
    sets = default_gang_sets(world, gpv, a.gang)
    times = prof.profile_models(a.models.split(","), sets)
    res = None
    if prof.rank == 0:
        res = CommProfiler.classify(times, a.threshold)
        res["_meta"] = {"virtual_nodes": a.virtual_nodes, "gang_sets": sets, "nic_gbps": a.nic_gbps,
                        "device": str(prof.device), "threshold": a.threshold}
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        save(a.out, res)
        print(json.dumps(res, indent=1, default=str))
    dist.barrier()
    return res


if __name__ == "__main__":
    main()
