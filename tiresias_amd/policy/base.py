"""Scheduling-policy interface.

A policy never touches the cluster. The engine (``engine/sim.py`` for the
simulator, ``executor/cluster_runtime.py`` for real GPUs) calls:

* ``on_arrival(job, now)`` when a job is submitted;
* ``update(active, now)`` after time advanced (demotion, promotion, ranks);
* ``order(active, now)`` -> priority order. Preemptive policies order ALL
  active jobs (the engine keeps the longest prefix that fits, preempts the
  rest); non-preemptive ones order PENDING jobs (the engine starts them in
  order; ``blocking`` stops at the first that does not fit = head-of-line;
  ``lookahead`` bounds how many are tried);
* ``select(ordered, free_gpus, now)`` optional custom admission (multi-DLAS);
* ``next_event(active, now)`` -> the next time the ordering may change on its
  own (a demotion threshold, a starvation promotion, a time-slice boundary);
* ``after_schedule(active, now)`` bookkeeping; ``preempt_now(active, now)``
  for policies that preempt on their own clock (Gandiva time slicing);
* ``on_finish(job, now)`` when a job completes.

``prior`` is a HISTORY sample of job GPU-service (the reference's Gittins
prior file, ``run_sim.py:1682-1707``); ``None`` means no history: policies
that need a service distribution learn it online from finished jobs.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

from ..core.job import Job

INF = float("inf")


class Policy:
    name = "base"
    preemptive = False
    blocking = False
    lookahead: Optional[int] = None
    default_placement = "yarn"

    def __init__(self, cfg=None, prior: Optional[List[float]] = None, rng=None):
        self.cfg = cfg
        self.prior = prior
        self.rng = rng
        self._seq = 0

    def next_seq(self) -> int:
        self._seq += 1
        return self._seq

    def on_arrival(self, job: Job, now: float) -> None:
        job.queue = 0
        job.extra["seq"] = self.next_seq()

    def update(self, active: List[Job], now: float) -> None:
        pass

    def order(self, active: List[Job], now: float) -> List[Job]:
        raise NotImplementedError

    def select(self, ordered: List[Job], free_gpus: int, now: float):
        return None

    def next_event(self, active: List[Job], now: float) -> float:
        return INF

    def after_schedule(self, active: List[Job], now: float) -> None:
        pass

    def preempt_now(self, active: List[Job], now: float) -> List[Job]:
        return []

    def on_finish(self, job: Job, now: float) -> None:
        """A job completed (policies with an online service prior learn here)."""


_REGISTRY: Dict[str, type] = {}


def register(*names):
    def deco(cls):
        for n in names:
            _REGISTRY[n] = cls
        return cls
    return deco


def make_policy(name: str, cfg=None, prior=None, rng=None) -> Policy:
    if name not in _REGISTRY:
        raise ValueError(f"unknown schedule {name!r}; choose from {sorted(_REGISTRY)}")
    p = _REGISTRY[name](cfg, prior=prior, rng=rng)
    p.name = name
    return p


def policies() -> List[str]:
    return sorted(_REGISTRY)


def submit_key(j: Job):
    try:
        jid = (0, int(j.job_id))
    except ValueError:
        jid = (1, j.job_id)
    return (j.spec.submit_time, jid)
