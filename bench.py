#!/usr/bin/env python
"""Headline benchmark: average JCT + makespan of a Tiresias-scheduled trace
replay on N MI355X GPUs (BASELINE.json metric).

One benchmark *step* = one complete replay of a fixed, seeded, Philly
(NSDI'19 Microsoft trace)-shaped job trace on the N GPUs of this node: real
training jobs (ResNet-50 / VGG-16 / Transformer-base / GNMT on the
hand-written gfx950 kernels, synthetic data, random init; multi-GPU jobs are
DDP gangs over RCCL) arrive over time, the Tiresias scheduler (discretized
2D-LAS on measured attained GPU service + skew-aware placement, HBM-resident
preemption, xGMI state moves) time-slices them, and every job trains its full
iteration budget. ``value`` is the average job completion time (seconds,
lower is better), ``makespan_s`` the replay makespan.

The trace is compressed so one replay takes a few seconds yet stays
scheduler-bound: ``--jobs-per-gpu`` (48) jobs per GPU with heavy-tailed
(log-normal) service times carrying ``--work-s`` GPU-seconds of nominal work
per GPU, arriving (Poisson) over work/``--load`` seconds, i.e. the offered
load exceeds capacity and a queue builds — the regime where the policy
decides JCT. Work scales with N (jobs per GPU fixed: weak scaling). The real
NSDI'19 trace is not shipped with the reference and there is no network, so
the trace is synthetic (``data`` says so).

Fairness of the comparison (``vs_baseline``): after the timed steps, the same
trace is replayed once under the reference's default FIFO + YARN-CS on the
same GPUs with the SAME sharing setting; ``vs_baseline`` = Tiresias avg JCT /
FIFO avg JCT (< 1 is better), the comparison BASELINE.md defines until the
real trace exists. The Gittins/expected-remaining prior, when a policy needs
one, comes from a held-out history trace (different seed), never from the
replayed jobs.

Time budget: the driver runs ``--steps 20 --warmup 5`` under a 600 s limit.
A guard (``--budget-s``, measured from process start) stops early — before a
step that would not fit — and the JSON line then reports the steps actually
timed (``steps`` < ``steps_requested``).

  python bench.py --gpus N --steps K --warmup W
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import time

T_PROC0 = time.perf_counter()

import argparse  # noqa: E402
import datetime  # noqa: E402
import gc  # noqa: E402
import json  # noqa: E402
import math  # noqa: E402
import os  # noqa: E402
import random  # noqa: E402
import statistics  # noqa: E402
import sys  # noqa: E402

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import faulthandler  # noqa: E402

# every rank: a fatal signal (SIGSEGV / SIGABRT / SIGBUS / SIGFPE) leaves all
# threads' Python stacks on stderr (round 4 recorded an undiagnosed rank-0
# SIGSEGV in the shared-GPU rehearsal)
faulthandler.enable(all_threads=True)
if os.environ.get("TAM_STACK_DUMP_S"):         # hang diagnosis: periodic all-thread stacks
    faulthandler.dump_traceback_later(float(os.environ["TAM_STACK_DUMP_S"]), repeat=True)

from tiresias_amd.config import ClusterSpec, SimConfig  # noqa: E402
from tiresias_amd.core.job import JobSpec  # noqa: E402
from tiresias_amd.executor.cluster_runtime import ReplayJob, Worker, run_replay  # noqa: E402

METRIC = "avg JCT + makespan on NSDI'19 Microsoft trace, 8×MI355X cluster"
MODEL_MIX = [("resnet50", 0.35), ("vgg16", 0.20), ("transformer", 0.30), ("gnmt", 0.15)]
TINY = {"resnet50": "resnet_tiny", "vgg16": "vgg_tiny", "transformer": "transformer_tiny",
        "gnmt": "gnmt_tiny"}
GPU_DIST = [(1, 0.70), (2, 0.12), (4, 0.10), (8, 0.08)]
# Frozen per-iteration seconds used ONLY to turn a sampled service time into an
# iteration count (round-1 measured MI355X hipGraph step times,
# profiles/model_bench_r1_v8.json). Kept constant so the benchmarked work
# (iterations per job) is identical across rounds: faster kernels then show
# up as lower JCT, not as a bigger trace.
SEQ_SCALE = 4
TRACE_ITER_S = {"resnet50": 0.0112, "vgg16": 0.0076, "transformer": 0.0068, "gnmt": 0.0153}
HISTORY_SEED_OFFSET = 7919          # the held-out history trace for the service prior
_routes_loaded = 0


def bench_trace(n_gpus: int, jobs_per_gpu: int, seed: int, work_s: float = 5.0, load: float = 1.6,
                sigma: float = 1.6, min_iters: int = 3, tiny: bool = False):
    """Philly-shaped compressed trace: ~70 % 1-GPU jobs with a power-of-two
    gang tail (gangs only when N allows), log-normal service (sigma 1.6: most
    jobs short, a few ~40x the median, as in the NSDI'19 trace) rescaled so
    the nominal GPU-work is ``work_s`` per GPU, Poisson arrivals over
    ``work_s / load`` seconds."""
    rng = random.Random(seed)
    n = jobs_per_gpu * n_gpus
    dist_ = [(g, p) for g, p in GPU_DIST if g <= n_gpus]
    tot = sum(p for _, p in dist_)
    gs, ps = [g for g, _ in dist_], [p / tot for _, p in dist_]
    names, ws = [m for m, _ in MODEL_MIX], [w for _, w in MODEL_MIX]
    rows = []
    for _ in range(n):
        m = rng.choices(names, weights=ws)[0]
        g = rng.choices(gs, weights=ps)[0]
        rows.append([m, g, rng.lognormvariate(0.0, sigma)])
    def it_s(m, g):
        return TRACE_ITER_S[m] * (1.0 if g == 1 else 1.1)

    def iters_of(scale):
        return [max(min_iters, int(round(x * scale / it_s(m, g)))) for m, g, x in rows]

    # rescale so the nominal work (after the min_iters clamp) is work_s per GPU
    target = work_s * n_gpus
    scale = target / sum(x * g for _, g, x in rows)
    for _ in range(8):
        w = sum(k * it_s(m, g) * g for k, (m, g, _) in zip(iters_of(scale), rows))
        scale *= target / w
    span = work_s / load
    rate = n / span
    jobs, t = [], 0.0
    for i, ((m, g, x), iters) in enumerate(zip(rows, iters_of(scale))):
        spec = JobSpec(job_id=str(i), submit_time=round(t, 4), duration=iters * it_s(m, g), num_gpu=g, model=m,
                       iterations=iters, gpu_util_avg=90.0, gpu_util_max=99.0)
        jobs.append(ReplayJob(spec=spec, model=TINY[m] if tiny else m, iterations=iters))
        t += rng.expovariate(rate)
    return jobs


def history_prior(jobs) -> list:
    """GPU-seconds of a held-out trace: the scheduler's service-time history."""
    return sorted(rj.spec.duration * rj.spec.num_gpu for rj in jobs)


def scenario_trace(name: str, n_gpus: int, seed: int, tiny: bool = False, sizes=None):
    """The other BASELINE.json configs as fixed job sets on the same runtime:

    * ``resnet4``  -- 4 concurrent ResNet-50 DDP jobs, each on n/4 GPUs (1
      GPU each when n < 4), all submitted at t=0 (config 2);
    * ``skew``     -- mixed ResNet-50 / VGG-16 multi-GPU gangs arriving
      together, so placement (consolidated vs spread) matters (config 3);
    * ``seq``      -- Transformer-base + GNMT jobs with staggered arrivals, for
      Gittins priority with preemption spilling state to host (config 4).
    """
    rng = random.Random(seed)
    rows = []
    if name == "resnet4":
        g = max(1, n_gpus // 4)
        rows = [("resnet50", g, 0.0, 60) for _ in range(4)]
    elif name == "skew":
        # sizes: the gang widths drawn uniformly (default 2 / 4 / 8; tools/
        # scenarios.py --sizes adds 1-GPU jobs, whose odd fragments are what
        # a spread decision can use on a 4x2 virtual-node split)
        sizes = [g for g in (sizes or (2, 4, 8)) if g <= n_gpus] or [1]
        t = 0.0
        for i in range(4 * n_gpus):
            m = "vgg16" if i % 2 else "resnet50"
            rows.append((m, rng.choice(sizes), round(t, 4), rng.choice((20, 40, 80))))
            t += rng.expovariate(4.0)
    elif name == "seq":
        # job sizes ~SEQ_SCALE x 12 iterations (0.3-3 s of GPU work): a spill +
        # restore of a GNMT job costs ~0.1 s of PCIe copies (profiles/r2/
        # preempt_costs.jsonl), so sub-second jobs would make every preemption
        # cost as much as the job; arrivals are stretched by the same factor
        t = 0.0
        for i in range(16 * n_gpus):
            m = "transformer" if i % 2 else "gnmt"
            g = rng.choice([g for g in (1, 1, 1, 2, 4) if g <= n_gpus])
            it = min(200, max(4, rng.lognormvariate(math.log(12), 1.2)))
            rows.append((m, g, round(t, 4), int(SEQ_SCALE * it)))
            t += rng.expovariate(16.0 / SEQ_SCALE)
    else:
        raise SystemExit(f"unknown scenario {name}")
    jobs = []
    for i, (m, g, t, iters) in enumerate(rows):
        spec = JobSpec(job_id=str(i), submit_time=t, duration=iters * TRACE_ITER_S[m], num_gpu=g,
                       model=m, iterations=iters, gpu_util_avg=90.0, gpu_util_max=99.0)
        jobs.append(ReplayJob(spec=spec, model=TINY[m] if tiny else m, iterations=iters))
    return jobs


# scenario -> (policy, placement, ckpt policy, baseline policy, baseline placement,
#              2D-LAS queue limits in GPU-seconds (resnet4 is "no preemption"),
#              GPU sharing when no GPU is free)
SCENARIOS = {
    "trace": ("dlas-gpu", "tiresias", "none", "fifo", "yarn", [0.05, 0.25, 1.0], False),
    "resnet4": ("dlas-gpu", "tiresias", "none", "fifo", "yarn", [1e9], False),
    "skew": ("dlas-gpu", "tiresias", "none", "dlas-gpu", "random", [1.0], False),
    "seq": ("gittins", "tiresias", "pressure", "fifo", "yarn", [0.2, 2.0], False),
}
# measured in-process co-run throughput of every model pair (tools/measure_stream_sharing.py)
SHARING_TABLE = os.path.join(ROOT, "profiles", "stream_sharing_mi355x.json")


def make_cfg(policy: str, scheme: str, n_gpus: int, seed: int, ckpt: str = "none",
             qlimits=(1.0,), share: bool = False, gittins_delta: float = 0.05, virtual_nodes: str = "",
             skew_profile: str = "") -> SimConfig:
    return SimConfig(schedule=policy, scheme=scheme, num_queue=len(qlimits) + 1, queue_limits=list(qlimits),
                     gittins_delta=gittins_delta, solve_starvation=0.0, seed=seed, ckpt_policy=ckpt,
                     virtual_nodes=virtual_nodes, skew_profile=skew_profile,
                     pack=share, max_tasks_per_gpu=2 if share else 3, gang_align=True,
                     interference_table=SHARING_TABLE if share else "",
                     cluster=ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=n_gpus,
                                         num_cpu_p_node=max(128, 16 * n_gpus),
                                         mem_p_node=max(512, 64 * n_gpus), gpu_memory_mb=288 * 1024))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scenario", default="trace", choices=sorted(SCENARIOS),
                    help="trace: the headline Philly-shaped replay; resnet4 / skew / seq: "
                         "BASELINE.json configs 2-4 (policy defaults follow the scenario)")
    ap.add_argument("--policy", default=None)
    ap.add_argument("--placement", default=None)
    ap.add_argument("--ckpt", default=None,
                    help="preemption state: none (stay in HBM) | pressure (spill to pinned host only when a "
                         "starting job needs the HBM) | host (always spill)")
    ap.add_argument("--hbm-budget-gb", type=float, default=None,
                    help="per-GPU HBM the jobs may use (pressure policy; default: the device's free HBM)")
    ap.add_argument("--baseline-policy", default=None)
    ap.add_argument("--baseline-placement", default=None)
    ap.add_argument("--no-baseline", action="store_true")
    ap.add_argument("--share", action="store_true",
                    help="co-locate 1-GPU jobs when the cluster is full (Tiresias AND baseline)")
    ap.add_argument("--jobs-per-gpu", type=int, default=48)
    ap.add_argument("--work-s", type=float, default=None,
                    help="nominal GPU-seconds of work per GPU per replay (default 5.0; 0.5 with --cpu)")
    ap.add_argument("--min-iters", type=int, default=3, help="shortest job, iterations")
    ap.add_argument("--virtual-nodes", default=None,
                    help="partition the node (e.g. 2x4); default: 2x(N/2) for --scenario skew at N>=4, "
                         "none otherwise. Spread gangs then pay the emulated inter-node link")
    ap.add_argument("--nic-gbps", type=float, default=12.5, help="emulated inter-virtual-node link, GB/s")
    ap.add_argument("--skew-profile", default="",
                    help="measured consolidated-vs-spread slowdowns (python -m tiresias_amd.profiler.comm)")
    ap.add_argument("--load", type=float, default=1.6, help="offered load / capacity during arrivals")
    ap.add_argument("--quantum", type=float, default=0.01,
                    help="scheduling round, seconds (0.01: N=1 avg JCT 0.1576 vs 0.1606 s at 0.02 on one "
                         "box, profiles/r5/quantum_ab.md; N>1 rounds end early anyway in fill mode)")
    ap.add_argument("--seed", type=int, default=2019)
    ap.add_argument("--budget-s", type=float, default=float(os.environ.get("TAM_BENCH_BUDGET_S", 270)),
                    help="wall budget from process start; steps that would not fit are skipped")
    ap.add_argument("--cpu", action="store_true", help="gloo/CPU rehearsal with tiny models")
    ap.add_argument("--no-graph", action="store_true",
                    help="disable hipGraph capture of 1-GPU jobs' fwd+bwd (eager launches)")
    ap.add_argument("--no-pool", action="store_true", help="no warm trainer reuse between jobs")
    ap.add_argument("--no-scale-limits", dest="scale_limits", action="store_false",
                    help="2D-LAS queue limits as given instead of per cluster GPU")
    ap.add_argument("--no-prewarm", action="store_true",
                    help="skip the per-process kernel pre-warm (one eager step per model family)")
    ap.add_argument("--no-nopool-replay", action="store_true",
                    help="skip the extra untimed replay without the warm pool (cold-build JCT)")
    ap.add_argument("--out", default=None, help="directory for job.csv / summary.json of the last step")
    ap.add_argument("--ddp-shard", action="store_true",
                    help="gangs: reduce-scatter + sharded optimizer + bf16 shadow all-gather (parallel/ddp.py)")
    ap.add_argument("--ddp-wire", default="fp32", choices=["fp32", "bf16"],
                    help="sharded gangs: reduce-scatter wire dtype")
    ap.add_argument("--preflight-s", type=float, default=120.0,
                    help="N > 1: bound of the communicator pre-flight (world + every canonical gang)")
    a = ap.parse_args()
    pol, plc, ck, bpol, bplc, qlim, share = SCENARIOS[a.scenario]
    share = share or a.share
    a.policy = a.policy or pol
    a.placement = a.placement or plc
    a.ckpt = a.ckpt or ck
    a.baseline_policy = a.baseline_policy or bpol
    a.baseline_placement = a.baseline_placement or bplc

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    n = max(a.gpus, world)
    use_cuda = torch.cuda.is_available() and not a.cpu
    work_s = a.work_s if a.work_s is not None else (5.0 if use_cuda else 0.5)
    # TAM_SHARED_GPU=1: multi-rank rehearsal on a ONE-GPU box -- every rank on
    # cuda:0, world and gang communicators over gloo (RCCL refuses two ranks
    # on one device); everything else is the N-GPU code path
    shared_gpu = use_cuda and world > 1 and os.environ.get("TAM_SHARED_GPU") == "1"
    device = torch.device("cuda", 0 if shared_gpu else local) if use_cuda else torch.device("cpu")
    ctrl_pg = world_pg = None
    if world > 1:
        from tiresias_amd.parallel.gang import configure_nccl_env

        configure_nccl_env()          # survivors of a lost rank must not be killed by the watchdog
        if shared_gpu:
            torch.cuda.set_device(device)
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
        elif use_cuda:
            torch.cuda.set_device(device)
            dist.init_process_group("nccl", device_id=device,
                                    timeout=datetime.timedelta(seconds=300))
        else:
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
        world_pg = dist.group.WORLD
        ctrl_pg = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=300))
        # warm the world communicator so later P2P / sub-groups do not need every rank
        tmp = torch.ones(1, device=device)
        dist.all_reduce(tmp)
    global _routes_loaded
    if use_cuda:
        from tiresias_amd.ops import _lib

        _lib.load(required=True)
        _routes_loaded = len([x for x in torch.ops.tam.gemm_routes().splitlines() if x.strip()])

    tiny = not use_cuda
    if a.scenario == "trace":
        jobs = bench_trace(n, a.jobs_per_gpu, a.seed, work_s=work_s, load=a.load, min_iters=a.min_iters,
                           tiny=tiny)
        prior = history_prior(bench_trace(n, a.jobs_per_gpu, a.seed + HISTORY_SEED_OFFSET,
                                          work_s=work_s, load=a.load, min_iters=a.min_iters))
    else:
        jobs = scenario_trace(a.scenario, n, a.seed, tiny=tiny)
        prior = history_prior(scenario_trace(a.scenario, n, a.seed + HISTORY_SEED_OFFSET))
    vn = a.virtual_nodes
    if vn is None:
        vn = f"2x{n // 2}" if (a.scenario == "skew" and n >= 4) else ""

    # 2D-LAS queue limits are GPU-seconds PER CLUSTER GPU: the thresholds
    # scale with the cluster's service rate (N GPU-s per second), so the
    # demotion / preemption rate per GPU stays what it is on one GPU as the
    # cluster grows. Unscaled, an N-GPU cluster preempts N times as often per
    # unit of work, and beyond one GPU a preemption often means a P2P state
    # move (fake backend, 10 seeds each, vs FIFO: N=2 0.58 -> 0.48, N=4
    # 0.49 -> 0.37, N=8 0.48 -> 0.32; N=1 unchanged)
    qlim_n = [x * n for x in qlim] if a.scale_limits else list(qlim)

    def make(policy, scheme, limits=None):
        # the Gittins quantum scales with the job sizes (a quantum below the
        # smallest prior job gives every new job index 0: no preemption)
        c = make_cfg(policy, scheme, n, a.seed, a.ckpt, qlim_n if limits is None else limits, share,
                     virtual_nodes=vn,
                     skew_profile=a.skew_profile,
                     gittins_delta=0.05 * (SEQ_SCALE if a.scenario == "seq" else 1))
        c.nic_gbps = a.nic_gbps
        c.ddp_shard, c.ddp_wire = a.ddp_shard, a.ddp_wire
        return c

    cfg = make(a.policy, a.placement)
    worker = Worker(rank, world, device, world_pg, use_graph=use_cuda and not a.no_graph,
                    gang_backend="gloo" if shared_gpu else None,
                    pool_cap=0 if a.no_pool else 2, hbm_budget_gb=a.hbm_budget_gb,
                    ddp_shard=a.ddp_shard, ddp_wire=a.ddp_wire)
    # per-process first-launch costs (kernel code objects, library handles),
    # paid once before the first replay like a cluster daemon's start-up
    prewarm_s = worker.prewarm(sorted({rj.model for rj in jobs})) if use_cuda and not a.no_prewarm else 0.0
    comm_setup_s = 0.0
    if world > 1:
        # gang_align placement puts every power-of-two gang on an aligned
        # buddy block: create (and warm) those communicators now, on every
        # rank in the same order, so no ncclCommInitRank lands in a replay
        from tiresias_amd.parallel.gang import canonical_gang_sets

        tc = time.perf_counter()
        vsz = int(vn.lower().split("x")[1]) if vn else 0
        worker.precreate_groups(canonical_gang_sets(n, vsz), vnode=vsz, nic_gbps=a.nic_gbps)
        worker.precreate_pairs()      # state-move communicators (one per rank pair)
        dist.barrier(group=ctrl_pg)
        comm_setup_s = time.perf_counter() - tc
        # pre-flight: known values all-reduced on the world communicator and
        # every canonical gang, checked exactly; any failure (wrong sum,
        # creation error, a member that never joins) stops EVERY rank with
        # the rank sets named, before anything is timed
        from tiresias_amd.parallel.gang import preflight

        errs = preflight(worker.groups, rank, device, world_pg, ctrl_pg, timeout_s=a.preflight_s)
        if errs:
            if rank == 0:
                for e in errs:
                    print(f"[bench] PREFLIGHT FAILED: {e}", file=sys.stderr, flush=True)
            os._exit(3)

    def sync():
        if world > 1:
            dist.barrier(group=ctrl_pg)
        if use_cuda:
            torch.cuda.synchronize(device)

    # Python's cyclic GC stays out of the replays: a gen-2 collection inside
    # one paused the controller for ~0.1 s (round 3's 0.2547 s outlier replay:
    # makespan +0.1 s with no eviction / spill / route change). Collected
    # between replays instead (untimed for the JCTs), with every long-lived
    # object frozen after the warm-up so those collections stay cheap; the
    # pause time of any collection that still happens is recorded per replay.
    gc_ms = [0.0]
    gc_t = [0.0]

    def _gc_cb(phase, info):
        if phase == "start":
            gc_t[0] = time.perf_counter()
        else:
            gc_ms[0] += (time.perf_counter() - gc_t[0]) * 1e3

    gc.callbacks.append(_gc_cb)
    replay_diag = []

    def replay(c, out=None):
        gc.collect()
        gc.disable()
        gc_ms[0] = 0.0
        ev0 = (worker.pool_evictions, worker.pressure_spills, worker.pool_hits)
        t = time.perf_counter()
        try:
            r = run_replay(c, jobs, rank, world, device, ctrl_pg=ctrl_pg, world_pg=world_pg,
                           worker=worker, quantum=a.quantum, out_dir=out, prior=prior)
        finally:
            gc.enable()
        dt = time.perf_counter() - t
        if r is not None:              # (the controller's summary lives on rank 0)
            replay_diag.append({"policy": f"{c.schedule}+{c.scheme}", "avg_jct": round(r["avg_jct"], 4),
                                "makespan": round(r["makespan"], 4), "wall_s": round(dt, 3),
                                "gc_ms": round(gc_ms[0], 2),
                                "pool_evictions": worker.pool_evictions - ev0[0],
                                "pressure_spills": worker.pressure_spills - ev0[1],
                                "pool_hits": worker.pool_hits - ev0[2],
                                "breakdown": r.get("runtime_breakdown")})
        if rank == 0:                  # progress on stderr (the JSON line stays alone on stdout)
            print(f"[bench] {c.schedule}+{c.scheme}{' share' if c.pack else ''}: avg JCT "
                  f"{r['avg_jct']:.4f} s, makespan {r['makespan']:.3f} s, {r['finished']} jobs, "
                  f"util {r['gpu_utilization']:.3f}, wall {dt:.2f} s (t={time.perf_counter() - T_PROC0:.0f}s)",
                  file=sys.stderr, flush=True)
        return r, dt

    def fits(longest: float) -> bool:
        """Every rank takes the same decision (rank 0's clock, broadcast)."""
        ok = torch.tensor([1 if time.perf_counter() - T_PROC0 + 1.25 * longest <= a.budget_s else 0])
        if world > 1:
            dist.broadcast(ok, 0, group=ctrl_pg)
        return bool(ok.item())

    longest = 0.0
    warm_done = 0
    cold = None
    for k in range(a.warmup):
        if k > 0 and not fits(longest):
            break
        r_, dt = replay(cfg)
        if k == 0:
            cold = r_             # the first replay of a fresh process: every trainer built cold
        longest = max(longest, dt)
        warm_done += 1
    gc.collect()
    gc.freeze()                       # warm-up state is long-lived: out of every later collection
    sync()
    t0 = time.perf_counter()
    sums = []
    walls = []
    for k in range(a.steps):
        if k > 0 and not fits(longest):
            break
        s, dt = replay(cfg, a.out if (a.out and k == a.steps - 1) else None)
        longest = max(longest, dt)
        sums.append(s)
        walls.append(dt)
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ctrl_pg)
        elapsed = float(t.item())
    steps = len(sums)

    base = None
    if not a.no_baseline and fits(3.0 * longest):
        # FIFO is non-preemptive: its replay can run longer than Tiresias'
        bcfg = make(a.baseline_policy, a.baseline_placement)
        base, _ = replay(bcfg)
    # the reference treats 2D-LAS queue limits as absolute GPU-seconds
    # (run_sim.py dlas_sim_jobs): one untimed replay with the UNSCALED limits
    # reports that reference-faithful number next to the headline (at N = 1
    # the two configurations are the same)
    unscaled = None
    if a.scale_limits and n > 1 and fits(1.5 * longest):
        unscaled, _ = replay(make(a.policy, a.placement, limits=list(qlim)))
    nopool = None
    if not a.no_pool and not a.no_nopool_replay and fits(1.5 * longest):
        # one replay WITHOUT the warm trainer pool: every job builds its own
        # trainer (allocation, init, eager warm-up, graph capture) inside its
        # JCT -- what a cluster pays when job shapes do not repeat
        cap = worker.pool_cap
        worker.drain_pool()
        worker.pool_cap = 0
        nopool, _ = replay(cfg)
        worker.pool_cap = cap

    # every rank's plan-application seconds by action kind over the whole
    # process (all replays), and its fill-mode steps: where N>1 time goes
    ap_all = [{"rank": rank, "apply_s": {k: round(v, 4) for k, v in sorted(worker.apply_prof.items())},
               "apply_n": dict(sorted(worker.apply_count.items())),
               "fill_s": round(worker.fill_s_total, 4), "fill_steps": worker.fill_steps_total}]
    if world > 1:
        got = [None] * world
        dist.all_gather_object(got, ap_all[0], group=ctrl_pg)
        ap_all = got
    if rank == 0:
        jcts = [s["avg_jct"] for s in sums]
        mks = [s["makespan"] for s in sums]
        avg_jct = statistics.fmean(jcts)
        makespan = statistics.fmean(mks)
        line = {
            "metric": METRIC,
            "value": round(avg_jct, 4),
            "unit": "s (avg JCT)",
            "n_gpus": n,
            "steps": steps,
            "warmup": warm_done,
            "ms_per_step": round(elapsed / steps * 1e3, 2),
            "higher_is_better": False,
            "scaling": "weak",
            "vs_baseline": round(avg_jct / base["avg_jct"], 4) if base else None,
            "dtype": "bf16",
            "data": "synthetic (Philly/NSDI'19-shaped compressed trace, random-init weights, synthetic batches)",
            "config": {
                "model": "mixed: resnet50 / vgg16 / transformer-base / gnmt jobs (DDP gangs when N>1)",
                "global_batch": "per job: per-GPU batch x gang size (64 img / 32 img / 32x128 tok / 64x50 tok)",
                "seq_len": "128 (transformer), 50 (gnmt)",
                "parallelism": f"dp (gang DDP over RCCL), {n} GPU cluster",
                "scenario": a.scenario,
                "ckpt": a.ckpt,
                "trace_jobs": len(jobs),
                "jobs_per_gpu": a.jobs_per_gpu,
                "work_gpu_s_per_gpu": work_s,
                "offered_load": a.load,
                "hip_graph_1gpu_jobs": bool(use_cuda and not a.no_graph),
                "warm_trainer_pool": not a.no_pool,
                "policy": f"{a.policy} + {a.placement} placement (Tiresias), queue limits {qlim} GPU-s"
                          + (f" per cluster GPU (= {qlim_n})" if a.scale_limits else "")
                          + (" + GPU sharing when full" if share else ""),
                "baseline": f"{a.baseline_policy} + {a.baseline_placement}"
                            + (" + GPU sharing when full" if share else ""),
                "prior": "held-out history trace (seed + %d)" % HISTORY_SEED_OFFSET,
                "quantum_s": a.quantum,
                "virtual_nodes": vn or None,
            },
            "steps_requested": a.steps,
            "warmup_requested": a.warmup,
            "makespan_s": round(makespan, 4),
            "avg_jct_per_step_s": [round(x, 4) for x in jcts],
            "avg_jct_stdev_s": round(statistics.stdev(jcts), 4) if len(jcts) > 1 else 0.0,
            "avg_jct_max_s": round(max(jcts), 4),
            "avg_jct_p95_s": round(sorted(jcts)[min(len(jcts) - 1, int(math.ceil(0.95 * len(jcts))) - 1)], 4),
            # per timed replay: GC pause inside it, pool / spill activity, and
            # the controller's runtime breakdown (outlier attribution)
            "replay_diag": replay_diag[warm_done:warm_done + steps],
            "makespan_per_step_s": [round(x, 4) for x in mks],
            "replay_wall_per_step_s": [round(x, 3) for x in walls],
            "median_jct_s": round(statistics.fmean(s["median_jct"] for s in sums), 4),
            "p95_jct_s": round(statistics.fmean(s["p95_jct"] for s in sums), 4),
            "preemptions": sums[-1]["preemptions"],
            "finished_jobs": sums[-1]["finished"],
            "baseline_avg_jct_s": round(base["avg_jct"], 4) if base else None,
            "unscaled_limits_avg_jct_s": (round(unscaled["avg_jct"], 4) if unscaled else
                                          (round(avg_jct, 4) if (n == 1 or not a.scale_limits) else None)),
            "unscaled_limits_vs_baseline": (round((unscaled["avg_jct"] if unscaled else avg_jct) / base["avg_jct"], 4)
                                            if base and (unscaled or n == 1 or not a.scale_limits) else None),
            # cold start, both untimed: the first warm-up replay of this fresh
            # process, and one replay with the warm trainer pool disabled
            "cold_first_replay_avg_jct_s": round(cold["avg_jct"], 4) if cold else None,
            "no_pool_replay_avg_jct_s": round(nopool["avg_jct"], 4) if nopool else None,
            "gemm_routes_preloaded": _routes_loaded,
            "baseline_makespan_s": round(base["makespan"], 4) if base else None,
            "shared_rounds": sums[-1].get("shared_rounds"),
            "gpu_utilization": round(statistics.fmean(s["gpu_utilization"] for s in sums), 4),
            "runtime_breakdown_s": sums[-1].get("runtime_breakdown"),
            "apply_breakdown_last_replay_rank0_s": sums[-1].get("apply_breakdown_rank0"),
            "apply_counts_last_replay_rank0": sums[-1].get("apply_counts_rank0"),
            "per_rank_process_totals": ap_all,
            "fill_mode": bool(worker.fill_enabled and world > 1),
            "comm_totals_last_replay_s": sums[-1].get("comm_totals_s"),
            "pool_hits": worker.pool_hits,
            "pressure_spills": worker.pressure_spills,
            "pool_evictions": worker.pool_evictions,
            "restore_prefetches": worker.prefetches,
            "replays": warm_done + steps + (1 if base else 0) + (1 if nopool else 0) + (1 if unscaled else 0),
            "comm_precreate_s": round(comm_setup_s, 3),
            "process_prewarm_s": round(prewarm_s, 3),
            "comm_stats": sums[-1].get("comm_stats"),
            "gang_errors": sum(s_.get("gang_errors", 0) for s_ in sums),
            "step_errors": [e for s_ in sums for e in s_.get("step_errors", [])][:10],
            "spilled_gb": round(worker.spilled_bytes / 2 ** 30, 3),
            "max_hbm_reserved_gb": round(torch.cuda.max_memory_reserved(device) / 2 ** 30, 2) if use_cuda else None,
            "process_wall_s": round(time.perf_counter() - T_PROC0, 1),
            "device": torch.cuda.get_device_name(device) if use_cuda else "cpu",
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier(group=ctrl_pg)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
