"""Discrete-event cluster simulator (and the reference-compatible tick loop).

Event engine (default). Time jumps to the next of: a trace arrival, the
earliest predicted job completion, or the policy's next self-triggered change
(2D-LAS demotion / starvation promotion, Gittins quantum, Gandiva time-slice,
multi-DLAS re-plan). At each event:

  1. advance every active job to ``now`` (progress, attained service,
     pending time);
  2. complete finished jobs (release resources, write job.csv);
  3. admit arrivals (``policy.on_arrival``);
  4. ``policy.update`` (demote / promote / re-rank);
  5. schedule: preemptive policies keep the longest priority prefix that
     fits (count feasibility, or ``policy.select``), preempt the rest, place
     pending members via the placement engine, then back-fill lower-priority
     pending jobs into idle GPUs (work conserving); non-preemptive policies
     start pending jobs in order (head-of-line ``blocking`` / ``lookahead``);
  6. plugins: policy time-slicing, migration;
  7. log cluster.csv + decisions.

Many jobs may be placed per event (the live reference places at most one per
tick, ``schedule.py:188-189``; ``TickSimulator`` keeps that behaviour for
cross-checks). The loop ends only when every job has finished or can never
run (defect D1: the reference stops while jobs are still queued). All
randomness is seeded (defect D10).

Tick engine (``engine="tick"``): the live Horus simulator's fixed-tick loop
(``core/scheduling/schedule.py:178-212``) — one tick per time unit, at most
``max_place_per_tick`` placements, progress +1 per tick x rate, Gandiva time
slices on processed-time multiples — defect-free.
"""
from __future__ import annotations

import math
import random
import time
from typing import Dict, List, Optional

from ..cluster.interference import InterferenceModel
from ..cluster.network import allreduce_seconds, measured_spread_rate, network_rate
from ..cluster.topology import Cluster, PlacementError
from ..config import SimConfig
from ..core.job import Job, JobSpec, JobState
from ..metrics.logger import MetricsLogger
from ..placement.schemes import align_plan, make_placement
from ..policy import make_policy
from ..profiler.skew import SensitivityOracle, model_profile
from ..trace.readers import StreamingReader
from .ckpt_model import CkptCostModel
from .spread import ServiceEstimate, SpreadAdvisor

EPS = 1e-9
PACK_SCHEMES = {"horus", "horus+", "gandiva", "pack"}


class Simulator:
    def __init__(self, cfg: SimConfig, specs: List[JobSpec], logger: Optional[MetricsLogger] = None,
                 prior: Optional[List[float]] = None, check_invariants: bool = False):
        self.cfg = cfg
        self.rng = random.Random(cfg.seed)
        scheme = cfg.scheme
        if scheme in ("", "default"):
            scheme = None
        self.policy = make_policy(cfg.schedule, cfg, prior=self._prior(specs, prior), rng=self.rng)
        scheme = scheme or self.policy.default_placement
        if cfg.schedule == "dlas-gpu-pack" and cfg.scheme in ("", "default", "yarn"):
            scheme = "pack"
        pack = cfg.pack or scheme in PACK_SCHEMES
        self.scheme = scheme
        self.cluster = Cluster(cfg.cluster, pack=pack, max_tasks_per_gpu=cfg.max_tasks_per_gpu,
                               headroom_mb=cfg.gpu_mem_headroom_mb, virtual_nodes=cfg.virtual_nodes)
        self.oracle = SensitivityOracle(cfg.skew_threshold, measured_path=cfg.skew_profile)
        self.placement = make_placement(scheme, rng=random.Random(cfg.seed + 1),
                                        sensitivity=self.oracle,
                                        cluster_gpus_per_node=self.cluster.spec.num_gpu_p_node,
                                        pack=pack)
        self.jobs: Dict[str, Job] = {}
        for s in specs:
            if s.job_id in self.jobs:
                raise ValueError(f"duplicate job id {s.job_id}")
            self.jobs[s.job_id] = Job(s)
        self.reader = StreamingReader(specs)
        self.log = logger or MetricsLogger(None)
        self.ckpt = CkptCostModel(cfg.ckpt_policy, cfg.ckpt_bw_gbps, cfg.ckpt_hbm_budget_gb,
                                  table_path=cfg.ckpt_table if cfg.ckpt_policy == "measured" else "")
        self.interf = (InterferenceModel.load(cfg.interference_table, cfg.interference)
                       if cfg.interference_table else InterferenceModel(cfg.interference))
        self.placement.model_of = lambda jid: self.jobs[jid].spec.model or ""
        self.placement.pair_cost = lambda a, b: self.interf.pair(a, b)
        # service-time history for non-clairvoyant remaining-time estimates
        # (the Gittins prior; learned from finished jobs when there is none)
        prior_s = self._prior(specs, prior)
        self._svc = ServiceEstimate(prior_s)
        self._svc_online = not prior_s
        # per-iteration seconds of a job (the live controller overrides it:
        # its job durations are iteration counts)
        self.iter_s_of = lambda j: (j.spec.duration / j.spec.iterations
                                    if j.spec.iterations and j.spec.iterations > 0 else 0.25)
        rule = getattr(cfg, "spread_rule", "node")
        if rule not in ("node", "wait", "fragments", "price"):
            raise ValueError(f"spread_rule must be node | wait | price | fragments, got {rule!r}")
        if scheme == "tiresias" and rule in ("wait", "node", "price"):
            self.placement.advisor = SpreadAdvisor(self._remaining_wall, self._spread_rate,
                                                   price_fragments=rule == "price")
            self.placement.jobs_by_id = self.jobs
            self.placement.spread_node_gangs = rule != "node"
        self.now = 0.0
        self.active: List[Job] = []
        self.finished: List[Job] = []
        self.check = check_invariants
        # preemption rule of preemptive policies: "lazy" (only what a chosen
        # job's placement needs, _schedule_lazy) or "eager" (every running job
        # outside the priority prefix, then backfill)
        # (topology placements; "count" keeps the eager rule: no fragmentation)
        self.lazy_preempt = getattr(cfg, "preempt_rule", "lazy") == "lazy" and self.scheme != "count"
        self.events = 0
        self._stall = 0
        self.wall_s = 0.0
        gpn = self.cluster.spec.num_gpu_p_node
        self.max_gpus = self.cluster.num_gpus
        self._gpn = gpn

    def _prior(self, specs, prior):
        """The service prior comes from HISTORY (reference ``run_sim.py:
        1682-1707`` reads ``yarn-gput1000.csv``, a different trace): an
        explicit sample, else ``cfg.gittins_prior`` (csv with a duration
        column), else None = learned online from finished jobs. The trace's
        own (future) distribution is used only on request
        (``cfg.prior_mode == "oracle"``) and is flagged in the summary."""
        self.prior_source = "explicit"
        if prior is not None:
            return list(prior)
        path = getattr(self.cfg, "gittins_prior", "")
        if path:
            from ..trace.readers import read_duration_prior

            self.prior_source = "file"
            return read_duration_prior(path)
        if getattr(self.cfg, "prior_mode", "online") == "oracle":
            self.prior_source = "oracle"
            return sorted(s.duration * s.num_gpu for s in specs)
        self.prior_source = "online"
        return None

    def submit(self, spec: JobSpec) -> Job:
        """Online job submission (live runtime's spool API): registers the job;
        it arrives at ``spec.submit_time`` through the normal arrival path."""
        if spec.job_id in self.jobs:
            raise ValueError(f"duplicate job id {spec.job_id}")
        j = Job(spec)
        self.jobs[spec.job_id] = j
        self.reader.add(spec)
        return j

    # ------------------------------------------------------------------ helpers
    def _remaining_wall(self, j: Job) -> Optional[float]:
        """Expected wall seconds job j still needs (engine/spread.py)."""
        rem = self._svc.remaining(j.attained(True))
        if rem is None:
            return None
        r = j.rate if (j.is_running and j.rate > 0) else 1.0
        return rem / max(1, j.num_gpu) / r + (j.restore_left if j.is_running else 0.0)

    def _spread_rate(self, j: Job, k: int) -> float:
        """Progress rate of job j as a gang over k nodes: the measured 2-node
        slowdown ring-scaled to k, else the analytic all-reduce over the
        inter-node link (the emulated NIC with virtual nodes)."""
        if k <= 1:
            return 1.0
        sd = self.oracle.slowdown(j.spec.model or "")
        if sd is not None:
            return measured_spread_rate(sd, k)
        if self.cfg.virtual_nodes:           # the emulated NIC between virtual nodes
            from ..parallel.gang import DEFAULT_NIC_LATENCY_S

            bw, lat = getattr(self.cfg, "nic_gbps", 12.5) * 1000.0, DEFAULT_NIC_LATENCY_S
        else:
            bw, lat = self.cluster.spec.bandwidth_mbps, self.cluster.spec.internode_latency
        try:
            mb = model_profile(j.spec.model).total_mb if j.spec.model else 100.0
        except KeyError:
            mb = 100.0
        c = self.iter_s_of(j)
        comm = allreduce_seconds(mb * 2 ** 20, k, bw, lat)
        return c / (c + comm) if c > 0 else 1.0

    def _rate(self, j: Job) -> float:
        r = 1.0
        nodes = self.cluster.nodes_of(j.job_id)
        if self.cfg.enable_network_costs and len(nodes) > 1:
            sd = self.oracle.slowdown(j.spec.model or "")
            if sd is not None:
                r *= measured_spread_rate(sd, len(nodes))
            else:
                r *= network_rate(j, len(nodes), self.cluster.spec.bandwidth_mbps,
                                  self.cluster.spec.internode_latency)
        if self.cluster.pack:
            nb = self.cluster.neighbours(j.job_id)
            if nb:
                r *= self.interf.rate(j.spec.model or "", [self.jobs[k].spec.model or "" for k in nb])
        return r

    def _start(self, j: Job, plan) -> None:
        alloc = self.cluster.commit(j, plan)
        restore, nbytes = self.ckpt.on_resume(j, alloc)
        j.start(self.now, alloc, rate=1.0, restore_cost=restore)
        j.ckpt_bytes += nbytes
        j.extra["run_start"] = self.now
        self.log.decision(self.now, "start", j.job_id, gpus=j.num_gpu, nodes=sorted(alloc, key=int),
                          queue=j.queue, restore=restore)

    def _preempt(self, j: Job, reason: str = "priority") -> None:
        save, nbytes = self.ckpt.on_preempt(j, j.allocation)
        self.cluster.release(j)
        j.preempt(self.now, save, nbytes)
        self.log.decision(self.now, "preempt", j.job_id, reason=reason, save=save)

    def _finish(self, j: Job) -> None:
        self.cluster.release(j)
        j.finish(self.now)
        if self._svc_online:
            self._svc.add(j.total_executed * j.num_gpu)
        self.ckpt.on_finish(j)
        self.policy.on_finish(j, self.now)
        self.active.remove(j)
        self.finished.append(j)
        self.log.job_row(self.now, j)
        self.log.decision(self.now, "finish", j.job_id, jct=j.jct)

    def _refresh_rates(self) -> None:
        for j in self.active:
            if j.is_running:
                nr = self._rate(j)
                if abs(nr - j.rate) > 1e-12:
                    j.rate = nr
                    self.log.network_row(self.now, j.job_id, len(self.cluster.nodes_of(j.job_id)), nr)

    # ------------------------------------------------------------------ scheduling
    def _try_place(self, j: Job) -> bool:
        if j.num_gpu > self.max_gpus:
            return False
        plan = self.placement.plan(self.cluster, j)
        if self.cfg.gang_align:
            plan = align_plan(self.cluster, j, plan)
        if plan is None:
            return False
        try:
            self._start(j, plan)
        except PlacementError:
            return False
        return True

    def schedule(self) -> None:
        pol = self.policy
        if pol.preemptive:
            ordered = pol.order(self.active, self.now)
            chosen = pol.select(ordered, self.cluster.free_gpus(), self.now)
            if chosen is None:
                chosen, used = [], 0
                for j in ordered:
                    if used + j.num_gpu <= self.max_gpus:
                        chosen.append(j)
                        used += j.num_gpu
            cset = set(id(j) for j in chosen)
            # GPU sharing (pack): the priority-ordered exclusive set above
            # always runs; lower-priority 1-GPU jobs may additionally share
            # GPUs, but give their slot back whenever a chosen job (e.g. a
            # gang) cannot be placed because of them
            extra: List[Job] = []
            if self.cluster.pack:
                slots = self.max_gpus * (self.cluster.max_tasks - 1)
                for j in ordered:
                    if len(extra) >= slots:
                        break
                    if id(j) not in cset and j.num_gpu == 1:
                        extra.append(j)
            keep = cset | set(id(j) for j in extra)
            if self.lazy_preempt and not self.cluster.pack and not self.cfg.replace_all:
                self._schedule_lazy(ordered, chosen, keep)
                pol.after_schedule(self.active, self.now)
                return
            for j in list(self.active):
                if j.is_running and id(j) not in keep:
                    self._preempt(j)
            if self.cfg.replace_all:
                # legacy Tiresias: re-place every runnable job each event
                for j in chosen:
                    if j.is_running:
                        self._preempt(j, reason="replace")
            for j in chosen:
                if j.is_pending and not self._try_place(j):
                    for x in reversed(extra):
                        if x.is_running:
                            self._preempt(x, reason="unshare")
                            if self._try_place(j):
                                break
            for j in extra:
                if j.is_pending:
                    self._try_place(j)
            # work-conserving back-fill
            if self.cluster.free_gpus() > 0 or self.cluster.pack:
                for j in ordered:
                    if j.is_pending and id(j) not in cset and (
                            self.cluster.pack or j.num_gpu <= self.cluster.free_gpus()):
                        self._try_place(j)
        else:
            ordered = pol.order(self.active, self.now)
            tried = 0
            for j in ordered:
                if pol.lookahead is not None and tried >= pol.lookahead:
                    break
                tried += 1
                if not self._try_place(j) and pol.blocking:
                    break
        pol.after_schedule(self.active, self.now)

    def _schedule_lazy(self, ordered: List[Job], chosen: List[Job], keep: set) -> None:
        """Preempt only what a chosen job's placement actually needs.

        The priority prefix (``chosen``) is computed by GPU count, but a
        topology placement can still fail for a chosen job (no consolidated
        block, or the wait-vs-spread rule prefers waiting). Preempting every
        lower-priority running job up front then suspends jobs whose GPUs
        nobody takes -- they are backfilled right back (measured on the
        priced 2000-job Philly trace, 64 GPUs: 79 % of tiresias' and 67 % of
        yarn's Gittins preemptions restarted at the same instant, each paying
        a checkpoint stall, and often on other GPUs). Here the victims
        (running, not chosen) are released TENTATIVELY -- the chosen jobs are
        placed with every victim's GPUs available, as in the eager rule --
        and the back-fill then walks the priority order as the eager rule's
        does, except that a victim whose devices are all still free is
        re-committed in place (it never stopped) instead of being preempted
        and restarted; only the others are preempted."""
        victims = [j for j in ordered if j.is_running and id(j) not in keep]
        held: Dict[str, list] = {}
        for v in victims:
            held[v.job_id] = self.cluster.placed[v.job_id]
            self.cluster.release(v)
        for j in chosen:
            if j.is_pending:
                self._try_place(j)
        # work-conserving back-fill in priority order, as the eager rule's:
        # a victim whose devices are all still free is re-committed there (it
        # never stopped); one that cannot be is preempted now and, like any
        # pending job, placed wherever it fits (a migration)
        cset = set(id(j) for j in chosen)
        for j in ordered:
            plan = held.pop(j.job_id, None)
            if plan is not None:
                if self.cluster.validate(j, plan) is None:
                    self.cluster.commit(j, plan)
                    continue
                self._preempt(j)
            if j.is_pending and id(j) not in cset and 0 < j.num_gpu <= self.cluster.free_gpus():
                self._try_place(j)

    def _migrate(self) -> None:
        """Move a task off an overloaded device when idle devices exist
        (reference ``schedule.py:62-93``, which never fires, defect D7)."""
        idle = [(n.node_id, d.device_id) for n in self.cluster.nodes.values() for d in n.devices
                if d.is_idle()]
        if not idle:
            return
        worst, load = None, 1
        for n in self.cluster.nodes.values():
            for d in n.devices:
                if len(d.tasks) > load:
                    worst, load = d, len(d.tasks)
        if worst is None:
            return
        t = max(worst.tasks.values(), key=lambda t: t.gpu_util_avg)
        j = self.jobs[t.job_id]
        if j.is_running:
            self._preempt(j, reason="migrate")
            self.log.decision(self.now, "migrate", j.job_id)

    # ------------------------------------------------------------------ main loop
    def _next_time(self) -> float:
        t = self.reader.next_time()
        for j in self.active:
            if j.is_running:
                t = min(t, self.now + j.time_to_finish())
        t = min(t, self.policy.next_event(self.active, self.now))
        return t

    def _advance(self, t: float) -> None:
        for j in self.active:
            j.advance(t)
        self.log.account(t, self.cluster.busy_gpus())
        self.now = t

    def step(self, t: float) -> None:
        self._advance(t)
        tol = 1e-9 * max(1.0, self.now)
        for j in [j for j in self.active if j.is_running and
                  (j.remaining <= EPS * max(1.0, j.spec.duration) or j.time_to_finish() <= tol)]:
            j.progress = j.spec.duration
            self._finish(j)
        # arrivals within the clock tolerance of now (run() snaps such events to now)
        for s in self.reader.release(self.now + max(EPS, tol)):
            j = self.jobs[s.job_id]
            j.arrive(self.now)
            j.last_check = self.now
            self.policy.on_arrival(j, self.now)
            self.active.append(j)
            self.log.decision(self.now, "arrive", j.job_id, gpus=j.num_gpu)
        self.policy.update(self.active, self.now)
        for j in self.policy.preempt_now(self.active, self.now):
            if j.is_running:
                self._preempt(j, reason="timeslice")
        if self.cfg.enable_migration:
            self._migrate()
        self.schedule()
        self._refresh_rates()
        self.log.account(self.now, self.cluster.busy_gpus())
        if self.check:
            self.cluster.check_invariants()
            self._check_jobs()
        pend = [j for j in self.active if j.is_pending]
        self.log.cluster_row(self.now, self.cluster, pend, len(self.active) - len(pend),
                             len(self.finished))
        self.events += 1

    def _check_jobs(self) -> None:
        used = 0
        for j in self.active:
            if j.is_running:
                used += j.num_gpu
                assert j.spec.submit_time <= self.now + EPS, "job ran before submit"
        assert used <= self.max_gpus or self.cluster.pack, "GPU over-subscription"

    def run(self, until: float = math.inf, max_events: int = 50_000_000) -> Dict:
        t0 = time.perf_counter()
        self.step(min(self.reader.next_time(), until) if self.reader.remaining() else 0.0)
        while self.events < max_events:
            if not self.active and self.reader.remaining() == 0:
                break
            t = self._next_time()
            if t == math.inf:
                # nothing can change any more: jobs that can never be placed
                for j in list(self.active):
                    if j.is_pending:
                        j.state = JobState.FAILED
                        self.active.remove(j)
                        self.finished.append(j)
                        self.log.decision(self.now, "failed", j.job_id, reason="unplaceable")
                break
            if t > until:
                self._advance(until)
                break
            if t <= self.now + 1e-9 * max(1.0, self.now):
                t = self.now
                self._stall += 1
                if self._stall > 10000:
                    raise RuntimeError(f"simulator made no progress at t={self.now} "
                                       f"(policy {self.cfg.schedule} keeps requesting events at now)")
            else:
                self._stall = 0
            self.step(t)
        self.wall_s = time.perf_counter() - t0
        return self.summary()

    def summary(self) -> Dict:
        return self.log.summary(list(self.jobs.values()), self.cluster.num_gpus, self.wall_s,
                                extra=dict(schedule=self.cfg.schedule, scheme=self.scheme,
                                           events=self.events, prior=self.prior_source))


class TickSimulator(Simulator):
    """Fixed-tick loop with the live reference's ordering of phases."""

    def __init__(self, *a, max_place_per_tick: int = 1, **kw):
        super().__init__(*a, **kw)
        self.max_place = max_place_per_tick

    def _try_place_limited(self):
        pol = self.policy
        ordered = pol.order(self.active, self.now)
        placed = tried = 0
        for j in ordered:
            if placed >= self.max_place:
                break
            if pol.lookahead is not None and tried >= pol.lookahead:
                break
            tried += 1
            if self._try_place(j):
                placed += 1
            elif pol.blocking:
                break
        pol.after_schedule(self.active, self.now)

    def run(self, until: float = math.inf, max_events: int = 50_000_000) -> Dict:
        t0 = time.perf_counter()
        tick = 0
        if self.policy.preemptive:
            raise ValueError("tick engine reproduces the live (non-preemptive) policies only")
        while tick < max_events and tick <= until:
            if not self.active and self.reader.remaining() == 0:
                break
            for s in self.reader.release(tick + EPS):
                j = self.jobs[s.job_id]
                j.arrive(float(tick))
                self.policy.on_arrival(j, float(tick))
                self.active.append(j)
            if any(j.is_pending for j in self.active):
                self._try_place_limited()
            self._refresh_rates()
            tick += 1
            self._advance(float(tick))
            for j in [j for j in self.active if j.is_running and j.remaining <= EPS * max(1.0, j.spec.duration)]:
                self._finish(j)
            for j in self.policy.preempt_now(self.active, self.now):
                if j.is_running:
                    self._preempt(j, reason="timeslice")
            pend = [j for j in self.active if j.is_pending]
            self.log.cluster_row(self.now, self.cluster, pend, len(self.active) - len(pend),
                                 len(self.finished))
            self.events += 1
            if not self.active and self.reader.remaining() and self.reader.next_time() > tick:
                tick = int(math.floor(self.reader.next_time()))
                self._advance(float(tick))
        self.wall_s = time.perf_counter() - t0
        return self.summary()


def simulate(cfg: SimConfig, specs: List[JobSpec], out_dir: Optional[str] = None,
             prior: Optional[List[float]] = None, check_invariants: bool = False) -> Dict:
    log = MetricsLogger(out_dir)
    if cfg.schedule == "gandiva-ns":
        from .gandiva_ns import GandivaNodeSetSim

        try:
            return GandivaNodeSetSim(cfg, specs, logger=log, tick=cfg.gandiva_tick,
                                     slice_s=cfg.gandiva_slice, mem_util=cfg.gandiva_mem_util).run()
        finally:
            log.close()
    cls = TickSimulator if cfg.engine == "tick" else Simulator
    sim = cls(cfg, specs, logger=log, prior=prior, check_invariants=check_invariants)
    try:
        return sim.run()
    finally:
        log.close()
