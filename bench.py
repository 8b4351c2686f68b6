#!/usr/bin/env python
"""Headline benchmark: average JCT + makespan of a Tiresias-scheduled trace
replay on N MI355X GPUs (BASELINE.json metric).

One benchmark *step* = one complete replay of a fixed, seeded, Philly
(NSDI'19 Microsoft trace)-shaped job trace on the N GPUs of this node: real
DDP training jobs (ResNet-50 / VGG-16 / Transformer-base / GNMT on the
hand-written gfx950 kernels, synthetic data, random init) arrive over time,
the Tiresias scheduler (discretized 2D-LAS on measured attained GPU service +
skew-aware placement, HBM-resident preemption, xGMI state moves) time-slices
them, and every job trains its full iteration budget. ``ms_per_step`` is
therefore the replay makespan; ``value`` is the average job completion time
(seconds, lower is better). Work scales with N (jobs per GPU fixed: weak
scaling). The real NSDI'19 trace is not shipped with the reference and there
is no network, so the trace is synthetic (``data`` says so).

After the timed steps (outside the timed region) the same trace is replayed
once under the reference's default FIFO + YARN-CS scheduler on the same GPUs:
``vs_baseline`` = Tiresias avg JCT / FIFO avg JCT (< 1 is better), the
comparison BASELINE.md defines until the real trace exists.

  python bench.py --gpus N --steps K --warmup W
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import datetime
import json
import math
import os
import random
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tiresias_amd.config import ClusterSpec, SimConfig  # noqa: E402
from tiresias_amd.core.job import JobSpec  # noqa: E402
from tiresias_amd.executor.cluster_runtime import ReplayJob, Worker, run_replay  # noqa: E402

METRIC = "avg JCT + makespan on NSDI'19 Microsoft trace, 8×MI355X cluster"
MODEL_MIX = [("resnet50", 0.35), ("vgg16", 0.20), ("transformer", 0.30), ("gnmt", 0.15)]
TINY = {"resnet50": "resnet_tiny", "vgg16": "vgg_tiny", "transformer": "transformer_tiny",
        "gnmt": "gnmt_tiny"}
GPU_DIST = [(1, 0.70), (2, 0.10), (4, 0.10), (8, 0.07), (16, 0.03)]
# Frozen per-iteration seconds used ONLY to turn a sampled service time into an
# iteration count (round-1 measured MI355X step times). Kept constant so the
# benchmarked work (iterations per job) is identical across rounds: faster
# kernels then show up as lower JCT, not as a bigger trace.
TRACE_ITER_S = {"resnet50": 0.028, "vgg16": 0.015, "transformer": 0.016, "gnmt": 0.037}


def bench_trace(n_gpus: int, jobs_per_gpu: int, seed: int, median_s: float = 0.3, sigma: float = 1.8,
                load: float = 1.3, tiny: bool = False):
    """Philly-shaped mini trace: ~70% 1-GPU jobs with a power-of-two gang
    tail, heavy-tailed log-normal service times (sigma 1.8, i.e. most jobs
    short, a few 25x longer, as in the NSDI'19 trace), Poisson arrivals at
    ``load`` x capacity. Durations are compressed to seconds."""
    rng = random.Random(seed)
    n = jobs_per_gpu * n_gpus
    dist_ = [(g, p) for g, p in GPU_DIST if g <= n_gpus]
    tot = sum(p for _, p in dist_)
    gs, ps = [g for g, _ in dist_], [p / tot for _, p in dist_]
    names, ws = [m for m, _ in MODEL_MIX], [w for _, w in MODEL_MIX]
    rows = []
    for i in range(n):
        m = rng.choices(names, weights=ws)[0]
        g = rng.choices(gs, weights=ps)[0]
        svc = min(15.0, max(0.2, rng.lognormvariate(math.log(median_s), sigma)))
        it_s = TRACE_ITER_S[m] * (1.0 if g == 1 else 1.1)
        iters = max(4, int(round(svc / it_s)))
        rows.append((m, g, svc, iters))
    mean_work = sum(svc * g for _, g, svc, _ in rows) / n
    rate = load * n_gpus / mean_work
    t = 0.0
    jobs = []
    for i, (m, g, svc, iters) in enumerate(rows):
        model = TINY[m] if tiny else m
        spec = JobSpec(job_id=str(i), submit_time=round(t, 4), duration=svc, num_gpu=g, model=m,
                       iterations=iters, gpu_util_avg=90.0, gpu_util_max=99.0)
        jobs.append(ReplayJob(spec=spec, model=model, iterations=iters))
        t += rng.expovariate(rate)
    return jobs


def scenario_trace(name: str, n_gpus: int, seed: int, tiny: bool = False):
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
        sizes = [g for g in (2, 4, 8) if g <= n_gpus] or [1]
        t = 0.0
        for i in range(4 * n_gpus):
            m = "vgg16" if i % 2 else "resnet50"
            rows.append((m, rng.choice(sizes), round(t, 4), rng.choice((20, 40, 80))))
            t += rng.expovariate(4.0)
    elif name == "seq":
        t = 0.0
        for i in range(4 * n_gpus):
            m = "transformer" if i % 2 else "gnmt"
            g = rng.choice([g for g in (1, 1, 1, 2, 4) if g <= n_gpus])
            rows.append((m, g, round(t, 4), int(min(400, max(8, rng.lognormvariate(math.log(40), 1.2))))))
            t += rng.expovariate(3.0)
    else:
        raise SystemExit(f"unknown scenario {name}")
    jobs = []
    for i, (m, g, t, iters) in enumerate(rows):
        spec = JobSpec(job_id=str(i), submit_time=t, duration=iters * TRACE_ITER_S[m], num_gpu=g,
                       model=m, iterations=iters, gpu_util_avg=90.0, gpu_util_max=99.0)
        jobs.append(ReplayJob(spec=spec, model=TINY[m] if tiny else m, iterations=iters))
    return jobs


# scenario -> (policy, placement, ckpt policy, baseline policy, baseline placement,
#              2D-LAS queue-0 limit in GPU-seconds (resnet4 is "no preemption"),
#              GPU sharing when no GPU is free)
SCENARIOS = {
    "trace": ("dlas-gpu", "tiresias", "none", "fifo", "yarn", 1.0, True),
    "resnet4": ("dlas-gpu", "tiresias", "none", "fifo", "yarn", 1e9, False),
    "skew": ("dlas-gpu", "tiresias", "none", "dlas-gpu", "random", 1.0, False),
    "seq": ("gittins", "tiresias", "host", "fifo", "yarn", 1.0, False),
}
# measured in-process co-run throughput of every model pair (tools/measure_stream_sharing.py)
SHARING_TABLE = os.path.join(ROOT, "profiles", "stream_sharing_mi355x.json")


def make_cfg(policy: str, scheme: str, n_gpus: int, seed: int, ckpt: str = "none",
             qlimit: float = 1.0, share: bool = False) -> SimConfig:
    return SimConfig(schedule=policy, scheme=scheme, num_queue=2, queue_limits=[qlimit], gittins_delta=1.0,
                     solve_starvation=0.0, seed=seed, ckpt_policy=ckpt, pack=share,
                     max_tasks_per_gpu=2 if share else 3,
                     interference_table=SHARING_TABLE if share else "",
                     cluster=ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=n_gpus,
                                         num_cpu_p_node=max(128, 16 * n_gpus),
                                         mem_p_node=max(512, 64 * n_gpus), gpu_memory_mb=288 * 1024))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scenario", default="trace", choices=sorted(SCENARIOS),
                    help="trace: the headline Philly-shaped replay; resnet4 / skew / seq: "
                         "BASELINE.json configs 2-4 (policy defaults follow the scenario)")
    ap.add_argument("--policy", default=None)
    ap.add_argument("--placement", default=None)
    ap.add_argument("--ckpt", default=None, help="preemption state policy: none (HBM) | host")
    ap.add_argument("--baseline-policy", default=None)
    ap.add_argument("--baseline-placement", default=None)
    ap.add_argument("--no-baseline", action="store_true")
    ap.add_argument("--no-share", action="store_true",
                    help="exclusive GPUs only (no co-location of 1-GPU jobs when the cluster is full)")
    ap.add_argument("--no-exclusive-ref", action="store_true",
                    help="skip the untimed exclusive-GPU Tiresias replay reported next to the result")
    ap.add_argument("--jobs-per-gpu", type=int, default=16)
    ap.add_argument("--quantum", type=float, default=0.1)
    ap.add_argument("--seed", type=int, default=2019)
    ap.add_argument("--cpu", action="store_true", help="gloo/CPU rehearsal with tiny models")
    ap.add_argument("--no-graph", action="store_true",
                    help="disable hipGraph capture of 1-GPU jobs' fwd+bwd (eager launches)")
    ap.add_argument("--out", default=None, help="directory for job.csv / summary.json of the last step")
    a = ap.parse_args()
    pol, plc, ck, bpol, bplc, qlim, share = SCENARIOS[a.scenario]
    share = share and not a.no_share
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
    device = torch.device("cuda", local) if use_cuda else torch.device("cpu")
    ctrl_pg = world_pg = None
    if world > 1:
        if use_cuda:
            torch.cuda.set_device(device)
            dist.init_process_group("nccl", device_id=device,
                                    timeout=datetime.timedelta(seconds=600))
        else:
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=600))
        world_pg = dist.group.WORLD
        ctrl_pg = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=600))
        # warm the world communicator so later P2P / sub-groups do not need every rank
        tmp = torch.ones(1, device=device)
        dist.all_reduce(tmp)
    if use_cuda:
        from tiresias_amd.ops import _lib

        _lib.load(required=True)

    if a.scenario == "trace":
        jobs = bench_trace(n, a.jobs_per_gpu, a.seed, tiny=not use_cuda)
    else:
        jobs = scenario_trace(a.scenario, n, a.seed, tiny=not use_cuda)
    cfg = make_cfg(a.policy, a.placement, n, a.seed, a.ckpt, qlim, share)
    worker = Worker(rank, world, device, world_pg, use_graph=use_cuda and not a.no_graph)

    def sync():
        if world > 1:
            dist.barrier(group=ctrl_pg)
        if use_cuda:
            torch.cuda.synchronize(device)

    def replay(c, out=None):
        t = time.perf_counter()
        r = run_replay(c, jobs, rank, world, device, ctrl_pg=ctrl_pg, world_pg=world_pg,
                       worker=worker, quantum=a.quantum, out_dir=out)
        if rank == 0:                  # progress on stderr (the JSON line stays alone on stdout)
            print(f"[bench] {c.schedule}+{c.scheme}{' share' if c.pack else ''}: avg JCT "
                  f"{r['avg_jct']:.4f} s, makespan {r['makespan']:.3f} s, {r['finished']} jobs, "
                  f"wall {time.perf_counter() - t:.1f} s", file=sys.stderr, flush=True)
        return r

    for _ in range(a.warmup):
        replay(cfg)
    sync()
    t0 = time.perf_counter()
    sums = []
    for k in range(a.steps):
        s = replay(cfg, a.out if (a.out and k == a.steps - 1) else None)
        sums.append(s)
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ctrl_pg)
        elapsed = float(t.item())

    base = None
    if not a.no_baseline:
        bcfg = make_cfg(a.baseline_policy, a.baseline_placement, n, a.seed, a.ckpt, qlim)
        base = replay(bcfg)
    excl = None
    if share and not a.no_exclusive_ref:
        # the same Tiresias policy without GPU sharing (how much sharing buys)
        excl = replay(make_cfg(a.policy, a.placement, n, a.seed, a.ckpt, qlim, False))

    if rank == 0:
        avg_jct = sum(s["avg_jct"] for s in sums) / len(sums)
        makespan = sum(s["makespan"] for s in sums) / len(sums)
        line = {
            "metric": METRIC,
            "value": round(avg_jct, 4),
            "unit": "s (avg JCT)",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 2),
            "higher_is_better": False,
            "scaling": "weak",
            "vs_baseline": round(avg_jct / base["avg_jct"], 4) if base else None,
            "dtype": "bf16",
            "data": "synthetic (Philly/NSDI'19-shaped trace, random-init weights, synthetic batches)",
            "config": {
                "model": "mixed: resnet50 / vgg16 / transformer-base / gnmt DDP jobs",
                "global_batch": "per job: per-GPU batch x gang size (64 img / 32 img / 32x128 tok / 64x50 tok)",
                "seq_len": "128 (transformer), 50 (gnmt)",
                "parallelism": f"dp (gang DDP over RCCL), {n} GPU cluster",
                "scenario": a.scenario,
                "ckpt": a.ckpt,
                "trace_jobs": len(jobs),
                "hip_graph_1gpu_jobs": bool(use_cuda and not a.no_graph),
                "jobs_per_gpu": a.jobs_per_gpu,
                "policy": f"{a.policy} + {a.placement} placement (Tiresias)"
                          + (" + GPU sharing when full" if share else ""),
                "baseline": f"{a.baseline_policy} + {a.baseline_placement}",
                "quantum_s": a.quantum,
            },
            "makespan_s": round(makespan, 4),
            "median_jct_s": round(sum(s["median_jct"] for s in sums) / len(sums), 4),
            "p95_jct_s": round(sum(s["p95_jct"] for s in sums) / len(sums), 4),
            "preemptions": sums[-1]["preemptions"],
            "finished_jobs": sums[-1]["finished"],
            "baseline_avg_jct_s": round(base["avg_jct"], 4) if base else None,
            "baseline_makespan_s": round(base["makespan"], 4) if base else None,
            "tiresias_exclusive_avg_jct_s": round(excl["avg_jct"], 4) if excl else None,
            "tiresias_exclusive_makespan_s": round(excl["makespan"], 4) if excl else None,
            "shared_rounds": sums[-1].get("shared_rounds"),
            "gpu_utilization": round(sums[-1]["gpu_utilization"], 4),
            "runtime_breakdown_s": sums[-1].get("runtime_breakdown"),
            "device": torch.cuda.get_device_name(device) if use_cuda else "cpu",
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier(group=ctrl_pg)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
