"""BASELINE.json config 3 ("mixed ResNet-50 / VGG-16 jobs with skew-profiled
placement, consolidated vs spread, over xGMI") at the scale it names, on
the FAKE backend (``executor/fake.py``): the live controller's code path
(policy, placement, preemption, P2P moves, gang communicator lifecycle)
against an in-process model of 8 ranks split into 2 virtual nodes of 4,
where a spread gang pays the emulated inter-node link on every step. Times
are VIRTUAL seconds (measured MI355X step times + the link model), not
wall time on hardware: the 1-GPU box cannot run an 8-rank skew replay.

For each seed: the same job set under Tiresias (skew-aware placement,
consolidating placement-sensitive VGG-16 gangs; ``tiresias+wait``: the
same with the wait-vs-spread rule of engine/spread.py) vs random placement
vs YARN (always consolidate), all under 2D-LAS. Output: mean +- stdev over
seeds and the per-seed ratios.

    python tools/scenarios.py [--seeds 12] [--out profiles/r4/skew_fake_world8.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=12)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--nic-gbps", type=float, default=12.5)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r4", "skew_fake_world8.json"))
    ap.add_argument("--schemes", default="tiresias+wait,tiresias,random,yarn")
    ap.add_argument("--vnodes", default="",
                    help="virtual-node split of the world, e.g. 4x2 (4 nodes of 2 GPUs); default 2x(world/2)")
    ap.add_argument("--sizes", default="2,4,8", help="gang widths drawn uniformly (e.g. 1,1,2,4,8)")
    ap.add_argument("--current-steps", action="store_true",
                    help="the fake world steps at this round's measured MI355X step times "
                         "(profiler/step_times.py) instead of the runtime's nominal table")
    a = ap.parse_args()
    import bench
    from tiresias_amd.executor.fake import run_fake

    vn = a.vnodes or f"2x{a.world // 2}"
    from tiresias_amd.profiler.step_times import MI355X_STEP_S
    iter_s = dict(MI355X_STEP_S) if a.current_steps else None
    res = {}
    for name in a.schemes.split(","):
        scheme, _, rule = name.partition("+")
        res[name] = []
        for seed in range(1, a.seeds + 1):
            sizes = tuple(int(x) for x in a.sizes.split(","))
            jobs = bench.scenario_trace("skew", a.world, seed, sizes=sizes)
            prior = bench.history_prior(bench.scenario_trace("skew", a.world, seed + bench.HISTORY_SEED_OFFSET,
                                                             sizes=sizes))
            cfg = bench.make_cfg("dlas-gpu", scheme, a.world, seed, qlimits=[1.0], virtual_nodes=vn)
            cfg.nic_gbps = a.nic_gbps
            cfg.spread_rule = rule or "fragments"
            s = run_fake(cfg, jobs, a.world, quantum=0.02, prior=prior, iter_s=iter_s)
            res[name].append({"seed": seed, "avg_jct": s["avg_jct"], "makespan": s["makespan"],
                                "preemptions": s["preemptions"], "p2p_gb": s["fake_stats"]["p2p_bytes"] / 1e9,
                                "oracle": s.get("oracle"), "spread_advice": s.get("spread_advice")})
    out = {"what": f"fake backend, {a.world} ranks as virtual nodes {vn}, gang widths {a.sizes}, "
                   f"spread-gang link {a.nic_gbps} GB/s, "
                   "2D-LAS, mixed ResNet-50 / VGG-16 gangs (bench.py scenario 'skew'); VIRTUAL seconds",
           "seeds": a.seeds, "runs": res, "summary": {}}
    base = [r["avg_jct"] for r in res["random"]] if "random" in res else None
    for scheme, rows in res.items():
        j = [r["avg_jct"] for r in rows]
        m = [r["makespan"] for r in rows]
        ratio = [x / b for x, b in zip(j, base)] if base else [0.0, 0.0]
        out["summary"][scheme] = {"avg_jct_mean": round(statistics.fmean(j), 4),
                                  "avg_jct_stdev": round(statistics.stdev(j), 4),
                                  "makespan_mean": round(statistics.fmean(m), 4),
                                  "vs_random_mean": round(statistics.fmean(ratio), 4),
                                  "vs_random_stdev": round(statistics.stdev(ratio), 4)}
        if rows and rows[0].get("oracle"):
            out["summary"][scheme]["oracle_flips"] = sum(r["oracle"]["flips"] for r in rows)
            out["summary"][scheme]["oracle_decisions"] = sum(r["oracle"]["sensitive"] + r["oracle"]["insensitive"]
                                                             for r in rows)
    if "yarn" in res:
        y = [r["avg_jct"] for r in res["yarn"]]
        for scheme, rows in res.items():
            per = [r["avg_jct"] / b for r, b in zip(rows, y)]
            out["summary"][scheme]["vs_yarn_per_seed"] = [round(x, 4) for x in per]
            out["summary"][scheme]["vs_yarn_mean"] = round(statistics.fmean(per), 4)
    print(json.dumps(out["summary"], indent=1))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
