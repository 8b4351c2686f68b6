"""BASELINE config 1: CPU trace-replay sweep on a >=10k-job Philly-shaped
trace over 64 GPUs (8 nodes x 8), FIFO/YARN vs SRTF / SRSF vs 2D-LAS vs
Gittins, with the Gittins prior learned from a SEPARATE (held-out) history
trace (reference ``run_sim.py:1682-1707`` reads ``yarn-gput1000.csv``).

Two engines:
* the Python event engine with real placement (``yarn`` consolidated and the
  skew-aware ``tiresias`` scheme) -- the full simulator;
* the native C++ core (``csrc/sched_core``) -- the same policies under the
  same yarn / tiresias placements (plus count), month-scale speed; every
  native row with a Python twin is cross-checked (``match``: identical
  avg JCT, preemptions and finished count).

Writes ``profiles/sweep10k/sweep.csv`` + ``sweep.md`` (table) + the run's
trace / prior descriptors.

    python tools/sweep_10k.py [--jobs 10000] [--load 1.2] [--workers 6]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import csv
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

POLICIES = [("fifo", "yarn"), ("shortest", "yarn"), ("shortest-gpu", "yarn"), ("dlas-gpu", "yarn"),
            ("dlas-gpu", "tiresias"), ("gittins", "yarn"), ("gittins", "tiresias"),
            ("dlas-gpu-gittins", "tiresias")]


def _cfg(schedule, scheme, prior_path, seed, ckpt="none", net=False, preempt_rule="lazy"):
    from tiresias_amd.config import ClusterSpec, SimConfig

    return SimConfig(schedule=schedule, scheme=scheme, num_queue=2, queue_limits=[3600.0],
                     gittins_delta=3250.0, gittins_prior=prior_path, seed=seed,
                     ckpt_policy=ckpt, enable_network_costs=net, preempt_rule=preempt_rule,
                     ckpt_table=os.path.join(ROOT, "profiles", "ckpt_mi355x.json"),
                     cluster=ClusterSpec(num_switch=1, num_node_p_switch=8, num_gpu_p_node=8))


def _trace(n, load, seed):
    from tiresias_amd.trace.synth import philly_like_trace

    return philly_like_trace(n, 64, load=load, seed=seed)


def _run(args):
    engine, schedule, scheme, n, load, seed, prior_path, ckpt, net, rule = args
    specs = _trace(n, load, seed)
    cfg = _cfg(schedule, scheme, prior_path, seed, ckpt, net, rule)
    t = time.perf_counter()
    if engine == "native":
        from tiresias_amd.engine.native import simulate_native

        s = simulate_native(cfg, specs)
        s.pop("per_job", None)
    else:
        from tiresias_amd.engine.sim import simulate

        s = simulate(cfg, specs)
    if engine != "native":
        s["ckpt_gb"] = (s.get("ckpt_bytes") or 0.0) / 1e9      # the native summary's unit
    keep = ("avg_jct", "median_jct", "p95_jct", "makespan", "avg_queueing_delay", "preemptions", "finished",
            "jobs", "prior", "ckpt_overhead_s", "ckpt_gb")
    out = {k: s.get(k) for k in keep}
    out.update(engine=engine, schedule=schedule, scheme=scheme, wall_s=round(time.perf_counter() - t, 2))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=10000)
    ap.add_argument("--load", type=float, default=1.2)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--workers", type=int, default=6)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "sweep10k"))
    ap.add_argument("--native-only", action="store_true", help="skip the (slow) Python event engine rows")
    ap.add_argument("--ckpt_policy", default="none",
                    help="preemption cost: none | host | hbm | measured (profiles/ckpt_mi355x.json) | pressure")
    ap.add_argument("--preempt_rule", default="lazy", help="lazy | eager (engine/sim.py::_schedule_lazy)")
    ap.add_argument("--enable_network_costs", action="store_true",
                    help="spread gangs progress at the network-limited rate (cluster/network.py)")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    # held-out history: a different seed of the same generator, GPU-service
    hist = _trace(a.jobs, a.load, a.seed + 7919)
    prior_path = os.path.join(a.out, "history_prior.csv")
    with open(prior_path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["duration"])
        for s in hist:
            w.writerow([round(s.duration * s.num_gpu, 3)])
    runs = []
    for sch, sc in POLICIES:
        runs.append(("native", sch, sc, a.jobs, a.load, a.seed, prior_path, a.ckpt_policy,
                     a.enable_network_costs, a.preempt_rule))
    for sch in ("fifo", "shortest", "shortest-gpu", "dlas-gpu", "gittins", "dlas-gpu-gittins"):
        runs.append(("native", sch, "count", a.jobs, a.load, a.seed, prior_path, a.ckpt_policy,
                     a.enable_network_costs, a.preempt_rule))
    if not a.native_only:
        for sch, sc in POLICIES:
            runs.append(("event", sch, sc, a.jobs, a.load, a.seed, prior_path, a.ckpt_policy,
                         a.enable_network_costs, a.preempt_rule))
    res = []
    with cf.ProcessPoolExecutor(max_workers=a.workers) as ex:
        for r in ex.map(_run, runs):
            print(json.dumps(r), flush=True)
            res.append(r)
    twin = {(r["schedule"], r["scheme"]): r for r in res if r["engine"] == "event"}
    for r in res:
        t = twin.get((r["schedule"], r["scheme"])) if r["engine"] == "native" else None
        r["match"] = "" if t is None else (
            "yes" if (abs(t["avg_jct"] - r["avg_jct"]) <= 1e-6 * max(1.0, t["avg_jct"])
                      and t["preemptions"] == r["preemptions"] and t["finished"] == r["finished"]) else "NO")
    keys = ["engine", "schedule", "scheme", "avg_jct", "median_jct", "p95_jct", "makespan",
            "avg_queueing_delay", "preemptions", "finished", "jobs", "prior", "ckpt_overhead_s", "ckpt_gb",
            "wall_s", "match"]
    with open(os.path.join(a.out, "sweep.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, keys)
        w.writeheader()
        w.writerows(res)
    base = {(r["engine"], r["scheme"] == "count"): r["avg_jct"] for r in res if r["schedule"] == "fifo"}
    priced = ("costs: ckpt_policy " + a.ckpt_policy + (" (profiles/ckpt_mi355x.json bandwidths)"
                                                       if a.ckpt_policy == "measured" else "")
              + ("; spread gangs at the network-limited rate (analytic ring all-reduce over the "
                 "reference's 1250 MB/s, 0.015 s links)" if a.enable_network_costs else "; network free"))
    lines = [f"# {a.jobs}-job Philly-shaped trace, 64 GPUs (8x8), load {a.load}, seed {a.seed}, "
             f"preemption rule {a.preempt_rule}",
             "", "Gittins prior: held-out history trace (seed + 7919), GPU-seconds; 2D-LAS threshold 3600 "
             "GPU-s; Gittins quantum 3250 GPU-s.", "", priced + ".", "",
             "vs FIFO: against FIFO + yarn of the same engine (count rows: FIFO + count). match: the "
             "native row reproduces the Python event engine's row (avg JCT, preemptions, finished).", "",
             "| engine | policy | placement | avg JCT (s) | vs FIFO | median JCT | p95 JCT | makespan | "
             "preemptions | ckpt stall (s, all jobs) | wall (s) | match |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in res:
        b = base.get((r["engine"], r["scheme"] == "count"))
        lines.append(f"| {r['engine']} | {r['schedule']} | {r['scheme']} | {r['avg_jct']:.0f} | "
                     f"{(r['avg_jct'] / b) if b else float('nan'):.3f} | {r['median_jct']:.0f} | {r['p95_jct']:.0f} | "
                     f"{r['makespan']:.0f} | {r['preemptions']} | {(r.get('ckpt_overhead_s') or 0):.0f} | "
                     f"{r['wall_s']} | {r['match']} |")
    with open(os.path.join(a.out, "sweep.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
