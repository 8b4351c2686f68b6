"""Model-skew profiles: the data Tiresias' placement rule needs.

Tiresias (NSDI'19 §4.3) consolidates only *placement-sensitive* jobs — models
whose gradient traffic is dominated by a few huge tensors (VGG, AlexNet), so a
spread gang is throttled by the slowest link. The reference keeps only raw
per-tensor MB lists for 9 CNNs (``/root/reference/core/models.py:8-26``) and
never applies the rule. Here:

* ``LEGACY_PROFILES`` — the reference models summarised (#tensors, total MB,
  largest MB), so traces naming them keep working;
* ``model_profile(name)`` — exact per-parameter gradient sizes of OUR models
  (ResNet-50, VGG-16, Transformer-base, GNMT), derived from the same arena
  layout the DDP bucketer reduces;
* ``skew`` = largest tensor / total; ``is_sensitive`` thresholds it, or uses a
  *measured* consolidated-vs-spread all-reduce slowdown from the RCCL
  profiler (``profiler/comm.py``) when one is loaded.
"""
from __future__ import annotations

import functools
import json
import os
from dataclasses import dataclass
from typing import Dict, List, Optional

# name: (#tensors, total gradient MB, largest tensor MB)   [SURVEY §2.4 table]
LEGACY_PROFILES = {
    "vgg19": (15, 547.1, 392.0), "vgg16": (12, 526.8, 392.0), "vgg11": (9, 506.5, 392.0),
    "alexnet": (7, 235.8, 144.0), "resnet152": (48, 149.6, 9.0), "resnet101": (35, 119.7, 9.0),
    "resnet50": (18, 80.6, 9.0), "inception4": (81, 132.8, 5.9), "inception3": (21, 56.6, 7.8),
}


@dataclass
class ModelProfile:
    name: str
    params: int
    tensors: List[float]          # MB per gradient tensor (fp32)
    total_mb: float
    largest_mb: float

    @property
    def skew(self) -> float:
        return self.largest_mb / self.total_mb if self.total_mb > 0 else 0.0

    def state_bytes(self, opt: str = "sgd") -> int:
        # master fp32 + bf16 shadow + optimizer state (1 or 2 fp32 buffers)
        return self.params * (4 + 2 + (4 if opt == "sgd" else 8))


class _ShapeArena:
    """Records parameter shapes without allocating (for profiling)."""

    def __init__(self):
        import torch

        self.device = torch.device("cpu")
        self.shapes = []
        self.token = None

    def add(self, name, shape, init="normal", std=0.02, decay=True, fp32_compute=False, store_grad=False):
        from ..ops.arena import Param

        p = Param(name=name, shape=tuple(shape))
        n = 1
        for s in shape:
            n *= int(s)
        p.numel = n
        self.shapes.append((name, n))
        return p


@functools.lru_cache(maxsize=None)
def model_profile(name: str) -> ModelProfile:
    from ..models import FAMILY, MODELS, make_model

    if name in MODELS:
        ar = _ShapeArena()
        make_model(name, ar)
        sizes = [n * 4 / 2 ** 20 for _, n in ar.shapes]
        return ModelProfile(name, sum(n for _, n in ar.shapes), sizes, sum(sizes), max(sizes))
    if name in LEGACY_PROFILES:
        k, tot, big = LEGACY_PROFILES[name]
        rest = (tot - big) / max(1, k - 1)
        return ModelProfile(name, int(tot * 2 ** 20 / 4), [big] + [rest] * (k - 1), tot, big)
    fam = FAMILY.get(name)
    if fam:
        return model_profile(fam)
    raise KeyError(f"no profile for model {name!r}")


class SensitivityOracle:
    """Decides placement sensitivity from measured slowdowns when available,
    else from the static skew."""

    def __init__(self, threshold: float = 0.5, measured_path: str = "", slowdown_threshold: float = 1.25):
        """``measured_path``: the JSON ``profiler/comm.py`` writes (per model:
        iteration-level slowdown when spread over the virtual-node boundary,
        and the profiler's verdict). Models it covers are classified from the
        measurement; others (and tiny test models, via their family) fall
        back to the static skew."""
        self.threshold = threshold
        self.slowdown_threshold = slowdown_threshold
        self.measured: Dict[str, float] = {}
        self.source = "static-skew"
        if measured_path:
            if not os.path.exists(measured_path):
                raise FileNotFoundError(f"skew profile {measured_path!r} not found "
                                        "(python -m tiresias_amd.profiler.comm writes it)")
            with open(measured_path) as f:
                data = json.load(f)
            for k, v in data.items():
                if k.startswith("_"):
                    continue
                self.measured[k] = float(v.get("slowdown", 1.0) if isinstance(v, dict) else v)
            self.source = measured_path

    def slowdown(self, model: str) -> Optional[float]:
        if model in self.measured:
            return self.measured[model]
        from ..cluster.interference import _TINY_BASE

        return self.measured.get(_TINY_BASE.get(model, ""))

    def __call__(self, job) -> bool:
        m = job.spec.model
        sd = self.slowdown(m)
        if sd is not None:
            return sd >= self.slowdown_threshold
        try:
            return model_profile(m).skew >= self.threshold
        except KeyError:
            return False
