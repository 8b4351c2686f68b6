"""Parameter sweeps over policies / placements / queue settings
(the reference's ``execute.py:5-57`` spawns one ``run_sim.py`` per setting
and polls every 5 s). Here runs execute in a process pool sized to the host,
each writes its own log directory, and a single ``sweep.csv`` collects the
summaries.

    python -m tiresias_amd.cli.sweep --synthetic 2000 \
        --schedules fifo,dlas-gpu,gittins --schemes yarn,tiresias --num_queues 2,3
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import csv
import itertools
import json
import os
import sys
import time


def _one(args):
    argv, tag = args
    from . import run_sim
    from ..config import FLAGS

    FLAGS.reset()
    s = run_sim.main(argv)
    s["tag"] = tag
    return s


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--schedules", default="fifo,dlas-gpu,dlas-gpu-gittins")
    ap.add_argument("--schemes", default="yarn")
    ap.add_argument("--num_queues", default="2")
    ap.add_argument("--repeats", type=int, default=1)
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 2))
    ap.add_argument("--out", default="log/sweep-" + time.strftime("%Y%m%d-%H%M%S"))
    a, rest = ap.parse_known_args(argv)
    runs = []
    for sch, sc, nq, rep in itertools.product(a.schedules.split(","), a.schemes.split(","),
                                             a.num_queues.split(","), range(a.repeats)):
        tag = f"{sch}_{sc}_q{nq}_r{rep}"
        argv1 = rest + ["--schedule", sch, "--scheme", sc, "--num_queue", nq, "--seed", str(rep),
                        "--log_path", os.path.abspath(os.path.join(a.out, tag))]
        runs.append((argv1, tag))
    os.makedirs(a.out, exist_ok=True)
    results = []
    with cf.ProcessPoolExecutor(max_workers=a.jobs) as ex:
        for s in ex.map(_one, runs):
            results.append(s)
            print(json.dumps({k: s[k] for k in ("tag", "avg_jct", "makespan", "finished")}), flush=True)
    keys = sorted({k for s in results for k in s})
    with open(os.path.join(a.out, "sweep.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, keys)
        w.writeheader()
        for s in results:
            w.writerow(s)
    return results


if __name__ == "__main__":
    main()
