"""Co-location interference model.

The reference models GPU sharing as one constant slowdown, ``FACTOR = 0.2``
(``infra/interference.py:1``), applied — in intent — to every co-located
task (``infra/node.py:189-204``; inert there, defect D-interference). Here the
slowdown is per (victim model, neighbour model) pair, MEASURED on MI355X by
``tools/measure_interference.py`` (two training processes time-sharing one
GPU; ``profiles/interference_mi355x.json``), with the constant as fallback
for pairs that were not measured.

``rate(model, neighbour_models)`` returns the progress-rate multiplier of a
job whose devices are shared with jobs of ``neighbour_models``: the worst
neighbour's measured slowdown s (step_time_colocated / step_time_alone) gives
rate = 1 / s.
"""
from __future__ import annotations

import json
from typing import Dict, Iterable, Optional, Tuple


_TINY_BASE = {"resnet_tiny": "resnet50", "vgg_tiny": "vgg16", "transformer_tiny": "transformer",
              "gnmt_tiny": "gnmt"}


class InterferenceModel:
    def __init__(self, default_factor: float = 0.2,
                 slowdown: Optional[Dict[Tuple[str, str], float]] = None, source: str = "constant"):
        self.default = 1.0 + float(default_factor)
        self.slowdown = dict(slowdown or {})
        self.source = source

    @staticmethod
    def load(path: str, default_factor: float = 0.2) -> "InterferenceModel":
        with open(path) as f:
            d = json.load(f)
        table = {}
        for key, v in d.get("slowdown", {}).items():
            a, b = key.split("|")
            table[(a, b)] = float(v)
        return InterferenceModel(default_factor, table, source=path)

    def pair(self, victim: str, neighbour: str) -> float:
        """Slowdown (>= 1) of ``victim`` co-located with ``neighbour``."""
        if (victim, neighbour) in self.slowdown:
            return self.slowdown[(victim, neighbour)]
        base = lambda m: _TINY_BASE.get(m, m)   # noqa: E731
        return self.slowdown.get((base(victim), base(neighbour)), self.default)

    def rate(self, victim: str, neighbours: Iterable[str]) -> float:
        ns = list(neighbours)
        if not ns:
            return 1.0
        return 1.0 / max(max(self.pair(victim, n) for n in ns), 1.0)

    def to_dict(self) -> Dict:
        return {"source": self.source, "default_slowdown": self.default,
                "slowdown": {f"{a}|{b}": v for (a, b), v in sorted(self.slowdown.items())}}
