"""Communication / skew profiler: measures the bucketed all-reduce a DDP gang
actually performs, on consolidated vs spread rank sets, and turns it into the
placement-sensitivity classification Tiresias' placement rule needs
(``profiler/skew.py::SensitivityOracle`` reads the JSON this writes).

On one 8x MI355X node every GPU pair has a direct xGMI link, so a gang's
all-reduce is (near) topology-insensitive; "spread" is emulated by the
virtual-node partition (``--virtual_nodes 2x4``): a spread gang crosses the
virtual-node boundary and, with ``spread_penalty_env`` set for the spread
communicator's process (e.g. ``NCCL_P2P_DISABLE=1`` -> shared-memory
transport), pays the slower path. Whatever the transport, the measurement —
not an assumption — decides sensitivity.

Run on N ranks (``torch.distributed`` initialised, RCCL on GPUs / gloo on
CPU)::

    prof = CommProfiler(dist.group.WORLD)
    res = prof.sweep([1, 4, 16, 64], gang_sets={"consolidated": [0,1,2,3], "spread": [0,4,1,5]})
    prof.classify_models(["resnet50", "vgg16"], res)  -> {"vgg16": {"slowdown": 1.3, ...}}
"""
from __future__ import annotations

import json
import time
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from .skew import model_profile


def ring_busbw(bytes_: float, seconds: float, n: int) -> float:
    """NCCL-convention bus bandwidth of an all-reduce (GB/s)."""
    if seconds <= 0 or n <= 1:
        return 0.0
    return bytes_ * 2 * (n - 1) / n / seconds / 1e9


class CommProfiler:
    def __init__(self, world_group=None, device: Optional[torch.device] = None, iters: int = 10,
                 warmup: int = 3):
        self.world = world_group
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.device = device or (torch.device("cuda", torch.cuda.current_device())
                                 if torch.cuda.is_available() else torch.device("cpu"))
        self.iters = iters
        self.warmup = warmup
        self._groups = {}

    def _group(self, ranks: Sequence[int]):
        key = tuple(sorted(ranks))
        if key not in self._groups:
            backend = "nccl" if self.device.type == "cuda" else "gloo"
            self._groups[key] = dist.new_group(list(key), backend=backend)   # collective on all ranks
        return self._groups[key]

    def time_allreduce(self, ranks: Sequence[int], nbytes: int) -> Optional[float]:
        g = self._group(ranks)
        if self.rank not in ranks:
            return None
        x = torch.ones(max(1, nbytes // 4), dtype=torch.float32, device=self.device)
        for _ in range(self.warmup):
            dist.all_reduce(x, group=g)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        for _ in range(self.iters):
            dist.all_reduce(x, group=g)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return (time.perf_counter() - t0) / self.iters

    def sweep(self, sizes_mb: Sequence[float], gang_sets: Dict[str, Sequence[int]]) -> Dict:
        """Returns {set_name: {size_mb: seconds}} (valid on member ranks)."""
        out: Dict[str, Dict[float, float]] = {}
        for name, ranks in gang_sets.items():
            self._group(ranks)
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

    @staticmethod
    def model_time(model: str, per_size: Dict[float, float], bucket_mb: float = 32.0) -> float:
        """Interpolated all-reduce time of a model's gradient buckets."""
        prof = model_profile(model)
        buckets, cur = [], 0.0
        for t in reversed(prof.tensors):
            cur += t
            if cur >= bucket_mb:
                buckets.append(cur)
                cur = 0.0
        if cur:
            buckets.append(cur)
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

    def classify_models(self, models: Sequence[str], sweep: Dict, threshold: float = 1.1) -> Dict:
        cons, spr = sweep.get("consolidated", {}), sweep.get("spread", {})
        out = {}
        for m in models:
            tc = self.model_time(m, cons)
            ts = self.model_time(m, spr)
            sd = ts / tc if tc > 0 else 1.0
            out[m] = {"consolidated_s": tc, "spread_s": ts, "slowdown": sd,
                      "skew": model_profile(m).skew, "sensitive": sd >= threshold}
        return out


def save(path: str, data: Dict) -> None:
    with open(path, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True, default=str)
