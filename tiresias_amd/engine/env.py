"""Gym-style environment over the simulator — the hook the reference stubs
(``/root/reference/model/env.py:1-7``, ``schedule.py:25-27`` "TODO: RL
agent").

Each ``step(action)`` picks which pending job to start next (index into the
current candidate list, or -1 to wait); the environment advances to the next
scheduling event and returns (observation, reward, done, info). Reward is the
negative number of active jobs integrated over the elapsed time, whose sum is
minus the total JCT — so maximising return minimises average JCT.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

from ..config import SimConfig
from ..core.job import JobSpec
from .sim import Simulator


class AgentPolicyEngine(Simulator):
    """Non-preemptive engine whose start decisions come from an agent."""

    def __init__(self, cfg: SimConfig, specs: List[JobSpec]):
        cfg = SimConfig(**{**cfg.__dict__, "schedule": "fjf"})
        super().__init__(cfg, specs)
        self.pending_action: Optional[int] = None

    def schedule(self) -> None:
        if self.pending_action is None or self.pending_action < 0:
            return
        cands = self.candidates()
        if self.pending_action < len(cands):
            self._try_place(cands[self.pending_action])
        self.pending_action = None

    def candidates(self):
        return sorted((j for j in self.active if j.is_pending), key=lambda j: j.spec.submit_time)


class SchedulingEnv:
    def __init__(self, cfg: SimConfig, specs: List[JobSpec], max_candidates: int = 8):
        self.cfg, self.specs, self.k = cfg, specs, max_candidates
        self.eng: Optional[AgentPolicyEngine] = None

    def _obs(self):
        e = self.eng
        c = e.candidates()[: self.k]
        feats = [[j.num_gpu, j.pending_time, j.spec.gpu_util_avg] for j in c]
        feats += [[0, 0, 0]] * (self.k - len(feats))
        return {"free_gpus": e.cluster.free_gpus(), "running": sum(1 for j in e.active if j.is_running),
                "candidates": feats, "now": e.now}

    def reset(self):
        self.eng = AgentPolicyEngine(self.cfg, self.specs)
        self.eng.step(self.eng.reader.next_time())
        return self._obs()

    def step(self, action: int) -> Tuple[dict, float, bool, dict]:
        e = self.eng
        e.pending_action = action
        before = e.now
        e.schedule()
        t = e._next_time()
        done = False
        if t == math.inf:
            done = not e.active and e.reader.remaining() == 0
            if not done:
                # no event will come: the agent must place something
                return self._obs(), -1.0, False, {"stalled": True}
        else:
            nactive = len(e.active)
            e.step(t)
            done = not e.active and e.reader.remaining() == 0
            return self._obs(), -(e.now - before) * nactive, done, {}
        return self._obs(), 0.0, done, {}
