"""GPU sharing inside ONE worker process: two jobs' steps interleaved on their
own HIP streams (what executor/cluster_runtime.py::Worker.run does for packed
jobs) vs the same steps run back to back. Reports, per model pair,
``speedup = (t_a + t_b) / t_together`` (> 1: co-running raises throughput)
and each job's slowdown, as JSON (the simulator's interference table format).

    python tools/measure_stream_sharing.py --steps 20 --out profiles/stream_sharing_mi355x.json
"""
import argparse
import itertools
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.executor.trainer import Trainer  # noqa: E402
from tiresias_amd.ops import _lib  # noqa: E402


def run(trainers, streams, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        for t, s in zip(trainers, streams):
            with torch.cuda.stream(s):
                t.step()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="resnet50,vgg16,transformer,gnmt")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    _lib.load(required=True)
    dev = torch.device("cuda", 0)
    models = a.models.split(",")
    tr = {}
    st = {}
    alone = {}
    for m in models:
        for k in (0, 1):                      # two instances (same-model pairs)
            t = Trainer(m, dev, seed=k, use_graph=True)
            s = torch.cuda.Stream(dev)
            run([t], [s], 4)                  # warm + capture
            tr[(m, k)], st[(m, k)] = t, s
        alone[m] = run([tr[(m, 0)]], [st[(m, 0)]], a.steps) / a.steps
        print(json.dumps({"model": m, "alone_ms": round(alone[m] * 1e3, 3)}), flush=True)
    res = {}
    for x, y in itertools.combinations_with_replacement(models, 2):
        ka, kb = (x, 0), (y, 1)
        tt = run([tr[ka], tr[kb]], [st[ka], st[kb]], a.steps) / a.steps
        seq = alone[x] + alone[y]
        r = {"alone_a_ms": round(alone[x] * 1e3, 3), "alone_b_ms": round(alone[y] * 1e3, 3),
             "together_ms": round(tt * 1e3, 3), "speedup": round(seq / tt, 4),
             # both jobs progress one step per `together` period
             "slowdown_a": round(tt / alone[x], 4), "slowdown_b": round(tt / alone[y], 4)}
        res[f"{x}|{y}"] = r
        print(json.dumps({f"{x}|{y}": r}), flush=True)
    if a.out:
        # simulator rate model: both co-located jobs progress at 1/s of their
        # solo speed with s = 2 / speedup (the pair's measured throughput)
        table = {}
        for k, r in res.items():
            x, y = k.split("|")
            table[f"{x}|{y}"] = table[f"{y}|{x}"] = round(2.0 / r["speedup"], 4)
        json.dump({"device": "MI355X, one process, per-job HIP streams", "steps": a.steps,
                   "slowdown": table, "raw": res}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
