"""Barrier idle of the bulk-synchronous live runtime at N = 2 / 4 / 8 on the
headline trace (bench.py's config), replayed through the real controller
against the fake backend in virtual time (executor/fake.py): per-rank idle at
the round's gather as a share of GPU time, by cause, with and without fill
mode. One JSON line per (N, fill, quantum); the mean over seeds.

    python tools/fake_barrier.py [--seeds 6] [--quanta 0.01] [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])

import bench  # noqa: E402
from tiresias_amd.executor.fake import FakeCluster, run_fake  # noqa: E402


def one(n, seed, fill, quantum, policy="dlas-gpu", scheme="tiresias"):
    jobs = bench.bench_trace(n, 48, seed)
    prior = bench.history_prior(bench.bench_trace(n, 48, seed + bench.HISTORY_SEED_OFFSET))
    cfg = bench.make_cfg(policy, scheme, n, seed, qlimits=[x * n for x in (0.05, 0.25, 1.0)])
    iters = dict(bench.TRACE_ITER_S)
    fc = FakeCluster(n, iter_s=iters, fill=fill)
    s = run_fake(cfg, jobs, n, quantum=quantum, prior=prior, iter_s=iters, fake=fc)
    st = s["fake_stats"]
    busy = st.get("busy_s", 0.0)
    idle = st.get("barrier_idle_s", 0.0)
    tot = busy + idle
    out = {"avg_jct": s["avg_jct"], "makespan": s["makespan"], "idle_frac": idle / tot if tot else 0.0}
    for k, v in st.items():
        if k.startswith("idle_"):
            out[k + "_frac"] = v / tot if tot else 0.0
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=6)
    ap.add_argument("--ns", default="2,4,8")
    ap.add_argument("--quanta", default="0.01")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    for n in [int(x) for x in a.ns.split(",")]:
        for q in [float(x) for x in a.quanta.split(",")]:
            for fill in (False, True):
                rs = [one(n, s, fill, q) for s in range(a.seeds)]
                keys = sorted({k for r in rs for k in r})
                row = {"n": n, "quantum": q, "fill": fill, "seeds": a.seeds}
                row.update({k: round(sum(r.get(k, 0.0) for r in rs) / len(rs), 4) for k in keys})
                rows.append(row)
                print(json.dumps(row), flush=True)
    if a.out:
        json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
