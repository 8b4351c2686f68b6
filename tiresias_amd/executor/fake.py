"""Fake (virtual-time) executor backend: ``--backend fake``.

The live runtime's CONTROLLER (``cluster_runtime.Controller``: the real
policy / placement / cluster objects, round planning, preemption decisions,
P2P donor selection, spill decisions) driven against an in-process model of
the N worker ranks instead of GPU processes (SURVEY §4 test plan item 4):

* every rank of the node lives in this one process; no torch.distributed, no
  GPU, no training — a round "runs" each rank's assignment by charging
  per-iteration times (measured MI355X step times, GPU-sharing slowdowns from
  the interference table, the spread-gang link penalty of
  ``parallel/gang.py``, state-move / spill / restore costs) to a
  ``VirtualClock``;
* it VALIDATES the scheduler<->executor protocol the real ``Worker`` relies
  on and raises ``ProtocolError`` on any violation: a gang started without
  its communicator, a "resident" resume on ranks that do not hold the state,
  P2P donors that hold nothing, a spill of a job that is not resident, a
  gang sharing a rank with another job (collectives would interleave), gang
  members assigned different step counts, a rank running a job it does not
  hold, a drop of an unknown job.

So the scheduler side of the live cluster (and the preemption state
machine) is testable at world 8+ in milliseconds, and a month-scale trace
can be replayed through the live controller's code path in virtual time.
"""
from __future__ import annotations

import math
import time
from typing import Dict, List, Optional, Set, Tuple

from ..config import SimConfig
from ..metrics.logger import MetricsLogger
from ..parallel.gang import ring_exchange_bytes, vnode_parts
from ..profiler.skew import model_profile
from .cluster_runtime import NOMINAL_ITER_S, Controller, ReplayJob


class ProtocolError(AssertionError):
    pass


class VirtualClock:
    def __init__(self, t0: float = 0.0):
        self.t = float(t0)

    def __call__(self) -> float:
        return self.t

    def advance(self, s: float) -> None:
        if s < 0:
            raise ValueError("virtual time cannot go backwards")
        self.t += s


def _state_bytes(model: str) -> float:
    from ..models import MODELS

    try:
        prof = model_profile(model)
    except KeyError:
        return 0.0
    opt = MODELS[model].opt if model in MODELS else "sgd"
    return float(prof.state_bytes(opt))


class FakeCluster:
    """N worker ranks in virtual time (see module docstring)."""

    def __init__(self, world: int, iter_s: Optional[Dict[str, float]] = None, interference=None,
                 vnode_size: int = 0, nic_gbps: float = 12.5, xgmi_gbps: float = 64.0,
                 host_gbps: float = 50.0, gang_factor: float = 1.08, start_s: float = 0.002,
                 fill: bool = True, vote_s: float = 60e-6):
        self.world = world
        self.iter_s = dict(NOMINAL_ITER_S)
        self.iter_s.update(iter_s or {})
        self.interf = interference
        self.vnode_size = vnode_size
        self.nic = nic_gbps * 1e9
        self.xgmi = xgmi_gbps * 1e9
        self.host = host_gbps * 1e9
        self.gang_factor = gang_factor
        self.start_s = start_s
        self.held: Dict[str, Tuple[int, ...]] = {}      # job -> ranks holding its state in HBM
        self.spilled: Set[str] = set()
        self.model: Dict[str, str] = {}
        self.groups: Set[Tuple[int, ...]] = set()
        self.stats = {"p2p_bytes": 0.0, "spill_bytes": 0.0, "restore_bytes": 0.0, "starts": 0,
                      "resident_resumes": 0, "rounds": 0}
        # fill mode (cluster_runtime.Worker.fill): a rank that finished its
        # round's share keeps stepping its job until the next plan arrives;
        # a gang agrees on every extra step with a one-element all-reduce
        # (vote_s). fill_seen: the fill steps the controller saw at plan time;
        # carry: steps completed after that (in flight when the plan came),
        # reported with the next round; late: how far into the next round a
        # rank's in-flight fill step runs
        self.fill = fill
        self.vote_s = vote_s
        self.fill_seen: Dict[str, int] = {}
        self.carry: Dict[int, Dict[str, Tuple[int, float]]] = {}
        self.late: Dict[int, float] = {}

    # ---------------------------------------------------------------- timing model
    def step_time(self, model: str, ranks: Tuple[int, ...]) -> float:
        t = self.iter_s.get(model, 0.03) * (1.0 if len(ranks) == 1 else self.gang_factor)
        parts = vnode_parts(ranks, self.vnode_size)
        if len(parts) > 1 and self.nic > 0:
            # spread gang: the gradient crosses the emulated inter-node link
            # every step (not hidden behind backward)
            grad = model_profile(model).params * 4.0
            t += ring_exchange_bytes(grad, len(parts)) / self.nic
        return t

    # ---------------------------------------------------------------- protocol
    def apply(self, plan: dict) -> Dict[int, float]:
        """Validate and cost the round's actions; returns per-rank seconds."""
        cost: Dict[int, float] = {}

        def charge(ranks, s):
            for r in ranks:
                cost[r] = cost.get(r, 0.0) + s

        for a in plan["actions"]:
            op, job = a["op"], a.get("job")
            if op == "group":
                ranks = tuple(a["ranks"])
                if len(ranks) < 2 or any(not 0 <= r < self.world for r in ranks):
                    raise ProtocolError(f"bad gang communicator {ranks}")
                if ranks in self.groups:
                    raise ProtocolError(f"communicator {ranks} created twice without ungroup/abort")
                self.groups.add(ranks)
                self.stats["comms_created"] = self.stats.get("comms_created", 0) + 1
                self.stats["peak_comms"] = max(self.stats.get("peak_comms", 0), len(self.groups))
            elif op in ("ungroup", "abort"):
                ranks = tuple(a["ranks"])
                if ranks not in self.groups:
                    raise ProtocolError(f"{op} of communicator {ranks} that does not exist")
                if op == "ungroup" and any(h == ranks for h in self.held.values()):
                    raise ProtocolError(f"ungroup of {ranks} while a job holds state on it")
                self.groups.discard(ranks)
            elif op == "drop":
                if job not in self.held:
                    raise ProtocolError(f"drop of job {job} that no rank holds")
                if tuple(a["ranks"]) != self.held[job]:
                    raise ProtocolError(f"drop of {job} on {a['ranks']} but held on {self.held[job]}")
                del self.held[job]
                self.spilled.discard(job)
            elif op == "consolidate":
                # a suspended sharded gang all-gathers its master / optimizer
                # slices over xGMI (parallel/ddp.py GradBucketer.consolidate)
                ranks = tuple(a["ranks"])
                if self.held.get(job) != ranks:
                    raise ProtocolError(f"consolidate of {job} on {ranks}, held on {self.held.get(job)}")
                if job in self.spilled:
                    raise ProtocolError(f"consolidate of {job} after its spill")
                w = len(ranks)
                b = _state_bytes(self.model[job]) * (w - 1) / w
                charge(ranks, b / self.xgmi)
                self.stats["consolidate_bytes"] = self.stats.get("consolidate_bytes", 0.0) + b * w
            elif op == "spill":
                if job not in self.held or job in self.spilled:
                    raise ProtocolError(f"spill of job {job} that is not resident")
                b = _state_bytes(self.model[job])
                charge(self.held[job], b / self.host)
                self.stats["spill_bytes"] += b * len(self.held[job])
                self.spilled.add(job)
            elif op == "start":
                ranks = tuple(a["ranks"])
                if len(ranks) > 1 and ranks not in self.groups:
                    raise ProtocolError(f"gang {job} started on {ranks} without a communicator")
                self.model[job] = a["model"]
                src = a["source"]
                b = _state_bytes(a["model"])
                if src == "fresh":
                    if job in self.held:
                        raise ProtocolError(f"fresh start of {job} whose state is still held")
                    charge(ranks, self.start_s)
                    self.stats["starts"] += 1
                elif src == "resident":
                    if self.held.get(job) != ranks:
                        raise ProtocolError(f"resident resume of {job} on {ranks}, held on {self.held.get(job)}")
                    self.stats["resident_resumes"] += 1
                    if job in self.spilled:
                        charge(ranks, b / self.host)
                        self.stats["restore_bytes"] += b * len(ranks)
                elif src == "p2p":
                    old = tuple(a["old"])
                    if self.held.get(job) != old:
                        raise ProtocolError(f"p2p move of {job} from {old}, held on {self.held.get(job)}")
                    donors = {int(k): int(v) for k, v in a["donors"].items()}
                    resync = bool(a.get("resync"))
                    for recv, donor in donors.items():
                        if donor not in old or recv not in ranks or (recv in old and not resync):
                            raise ProtocolError(f"bad donor {donor}->{recv} for {job}")
                    if resync:
                        if len(set(donors.values())) != 1 or set(ranks) - set(donors) - set(donors.values()):
                            raise ProtocolError(f"resync of {job} must copy ONE replica to every other member")
                    elif set(ranks) - set(old) != set(donors):
                        raise ProtocolError(f"new ranks of {job} without a donor")
                    if job in self.spilled:                  # holders restore first
                        charge(old, b / self.host)
                        self.stats["restore_bytes"] += b * len(old)
                    for recv, donor in donors.items():
                        charge((recv, donor), b / self.xgmi)
                        self.stats["p2p_bytes"] += b
                elif src == "snapshot":
                    # restart of a job whose every replica died: every member
                    # reads the last durable snapshot from host storage
                    if job in self.held:
                        raise ProtocolError(f"snapshot restart of {job} whose state is still held")
                    charge(ranks, b / self.host)
                    self.stats["restore_bytes"] += b * len(ranks)
                else:
                    raise ProtocolError(f"unknown start source {src}")
                self.held[job] = ranks
                self.spilled.discard(job)
            else:
                raise ProtocolError(f"unknown action {op}")
        return cost

    def run(self, plan: dict, now_abs: float, action_cost: Dict[int, float]):
        """One round: per-rank reports and the round's duration (the slowest
        rank; the real round ends with a gather over all ranks)."""
        assign = {int(r): list(v) for r, v in plan["assign"].items()}
        gang_n: Dict[str, int] = {}
        for r, lst in assign.items():
            for jid, n in lst:
                ranks = self.held.get(jid)
                if ranks is None or r not in ranks:
                    raise ProtocolError(f"rank {r} assigned job {jid} it does not hold")
                if jid in self.spilled:
                    raise ProtocolError(f"job {jid} assigned while spilled")
                if len(ranks) > 1:
                    if len(lst) > 1:
                        raise ProtocolError(f"gang {jid} shares rank {r} (collectives would interleave)")
                    if gang_n.setdefault(jid, n) != n:
                        raise ProtocolError(f"gang {jid} members assigned different step counts")
        deadline = plan.get("deadline")
        reports, busy = [], {}
        steps: Dict[int, float] = {}              # rank -> step seconds of its single job
        late = self.late
        self.late = {}
        left_of = plan.get("left") or {}
        # fill steps completed after the last plan snapshot are credited with
        # this round's reports, so the plan's share + left count them twice:
        # cap both by the carry (cluster_runtime.Worker.run)
        carried, self.carry = self.carry, {}
        fill_cap: Dict[str, int] = {}
        for r, lst in assign.items():
            if len(lst) == 1:
                jid, n = lst[0]
                c = sum(k for j2, (k, _) in (carried.get(r) or {}).items() if j2 == jid)
                if c > 0 and jid in left_of:
                    rem = int(left_of[jid]) + int(n) - c
                    n2 = max(0, min(int(n), rem))
                    fill_cap[jid] = max(0, rem - n2)
                    assign[r] = [(jid, n2)]

        def ready(x):
            return action_cost.get(x, 0.0) + late.get(x, 0.0)

        for r in range(self.world):
            lst = assign.get(r) or []
            t0 = ready(r)
            reps = []
            if len(lst) == 1:
                jid, n = lst[0]
                st = self.step_time(self.model[jid], self.held[jid])
                if len(self.held[jid]) > 1:
                    # a gang steps together: its members start when the last one is ready
                    t0 = max(ready(x) for x in self.held[jid])
                if deadline is not None and len(self.held[jid]) == 1 and n > 0:
                    # 1-GPU job: the round ends at the first step boundary after
                    # the next arrival (Worker._run_until)
                    left = deadline - (now_abs + t0)
                    n = max(1, min(n, int(math.floor(left / st)) + 1)) if left > 0 else 1
                busy[r] = t0 + n * st
                steps[r] = st
                reps.append({"job": jid, "iters": n, "run_s": n * st, "shared": False, "loss": None})
            elif lst:
                # co-located 1-GPU jobs run concurrently, each slowed by its partner
                ms = {jid: self.model[jid] for jid, _ in lst}
                dur = 0.0
                for jid, n in lst:
                    s = 1.0
                    if self.interf is not None:
                        s = max(self.interf.pair(ms[jid], ms[o]) for o in ms if o != jid)
                    dur = max(dur, n * self.step_time(ms[jid], (r,)) * s)
                busy[r] = t0 + dur
                for jid, n in lst:
                    reps.append({"job": jid, "iters": n, "run_s": dur, "shared": True, "loss": None})
            else:
                busy[r] = t0
            # fill steps completed after the last plan snapshot, in flight then
            for jid, (k, sec) in (carried.pop(r, None) or {}).items():
                reps.append({"job": jid, "iters": k, "run_s": sec, "shared": False, "loss": None, "fill": True})
            reports.append({"rank": r, "job": lst[0][0] if lst else None, "jobs": reps, "dev": None})
        self.stats["rounds"] += 1
        dur = max(busy.values()) if busy else 0.0
        # fill: ranks whose single job has iterations left keep stepping it
        # until the plan (at dur); a gang by agreement (vote per extra step)
        self.fill_seen = {}
        filled: Dict[int, float] = {}
        if self.fill:
            done_g: Dict[str, Tuple[int, int, float]] = {}
            for r in sorted(steps):
                jid, n = assign[r][0]
                ranks = self.held[jid]
                left = int(left_of.get(jid, 0))
                if jid in fill_cap:
                    left = min(left, fill_cap[jid])
                if left <= 0:
                    continue
                if len(ranks) > 1:
                    if jid not in done_g:
                        st = steps[r] + self.vote_s
                        b = max(busy[x] for x in ranks)
                        gap = dur - b
                        k = min(left, int(math.floor(gap / st))) if gap > 0 else 0
                        fl = 1 if (k < left and gap > 0) else 0       # the step in flight at the plan
                        done_g[jid] = (k, fl, st)
                    k, fl, st = done_g[jid]
                    b = max(busy[x] for x in ranks)
                else:
                    st = steps[r]
                    b = busy[r]
                    gap = dur - b
                    k = min(left, int(math.floor(gap / st))) if gap > 0 else 0
                    fl = 1 if (k < left and gap > 0) else 0
                if k:
                    self.fill_seen[jid] = k
                filled[r] = k * st
                if fl:
                    self.carry.setdefault(r, {})[jid] = (1, st)
                    self.late[r] = b + (k + 1) * st - dur
                    filled[r] = dur - b
        # barrier idle: a rank that had work this round but finished before
        # the slowest rank waits at the round's gather (bulk-synchronous
        # rounds) unless it fills; GPU time = what ranks with work were busy
        for r in assign:
            if assign[r]:
                self.stats["busy_s"] = self.stats.get("busy_s", 0.0) + busy[r] + filled.get(r, 0.0)
                idle = dur - busy[r] - min(filled.get(r, 0.0), dur - busy[r])
                self.stats["barrier_idle_s"] = self.stats.get("barrier_idle_s", 0.0) + idle
                jid = assign[r][0][0]
                why = ("shared" if len(assign[r]) > 1 else "job_done" if int(left_of.get(jid, 0)) <= 0
                       else "gang" if len(self.held[jid]) > 1 else "one_gpu")
                self.stats["idle_" + why] = self.stats.get("idle_" + why, 0.0) + idle
                self.stats["fill_s"] = self.stats.get("fill_s", 0.0) + filled.get(r, 0.0)
        return reports, dur


def run_fake(cfg: SimConfig, jobs: List[ReplayJob], world: int, quantum: float = 0.25,
             out_dir: Optional[str] = None, prior: Optional[List[float]] = None,
             iter_s: Optional[Dict[str, float]] = None, plan_cost_s: float = 0.0,
             max_rounds: int = 10 ** 8, fake: Optional[FakeCluster] = None,
             fill_rounds: bool = True) -> Dict:
    """Replay ``jobs`` through the live controller against a FakeCluster in
    virtual time. ``plan_cost_s`` charges each round's scheduling overhead."""
    from ..cluster.interference import InterferenceModel

    clock = VirtualClock()
    log = MetricsLogger(out_dir, node_logs=False)
    ctrl = Controller(cfg, jobs, world, quantum, logger=log, prior=prior, clock=clock)
    interf = (InterferenceModel.load(cfg.interference_table, cfg.interference)
              if cfg.interference_table else InterferenceModel(cfg.interference))
    fc = fake or FakeCluster(world, iter_s=iter_s, interference=interf, vnode_size=ctrl.vnode_size,
                             nic_gbps=ctrl.nic_gbps)
    ctrl.fill_rounds = fc.fill and fill_rounds
    if getattr(cfg, "gang_align", False):
        # the live bench pre-creates the canonical (buddy) communicators
        from ..parallel.gang import canonical_gang_sets

        sets = canonical_gang_sets(world, ctrl.vnode_size)
        ctrl.comms.pin(sets, ctrl.vnode_size)
        fc.groups.update(tuple(x) for x in sets)
    ctrl.start_clock()
    t_wall = time.perf_counter()
    rounds = 0
    while rounds < max_rounds:
        plan = ctrl.plan_round()
        cost = fc.apply(plan)
        if plan["stop"]:
            break
        reps, dt = fc.run(plan, clock(), cost)
        if not any(r["jobs"] for r in reps):
            dt = max(dt, plan.get("wait", 0.0))
            if dt <= 0.0:
                dt = 1e-6
        clock.advance(dt + plan_cost_s)
        ctrl.apply_reports(reps)
        if fc.fill_seen:
            ctrl.apply_fill(fc.fill_seen)     # read at plan time (live: the fill keys)
        rounds += 1
    if fc.held:
        raise ProtocolError(f"replay ended with state still held for {sorted(fc.held)}")
    s = ctrl.sched.summary()
    s.update(rounds=rounds, backend="fake", replay_wall_s=time.perf_counter() - t_wall, fake_stats=dict(fc.stats),
             virtual_s=clock(), comm_stats=dict(ctrl.comms.stats, live=len(ctrl.comms.live)),
             overrun_iters=ctrl.max_overrun, oracle=dict(getattr(ctrl.sched.placement, "oracle_stats", {})),
             spread_advice=dict(getattr(getattr(ctrl.sched.placement, "advisor", None), "decisions", {}) or {}))
    log.close()
    return s
