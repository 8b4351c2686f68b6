"""Measure GPU co-location interference on MI355X.

Two training processes (one per model of a pair) share ONE GPU, as the
``pack`` placement / Gandiva time-sharing would co-locate them. Each process
first times its step alone (the other waits at a barrier), then both run
together; slowdown = t_together / t_alone per victim. Output (JSON) feeds
``cluster.interference.InterferenceModel`` via ``--interference_table``.

usage: python tools/measure_interference.py --out profiles/interference_mi355x.json
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _proc(idx, model, steps, warmup, barrier, q):
    import torch

    from tiresias_amd.executor.trainer import Trainer
    from tiresias_amd.ops import _lib

    _lib.load(required=True)
    dev = torch.device("cuda", 0)
    t = Trainer(model, dev, seed=idx)
    for _ in range(warmup):
        t.step()
    torch.cuda.synchronize(dev)

    def timed():
        t0 = time.perf_counter()
        for _ in range(steps):
            t.step()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / steps

    alone = None
    for turn in range(2):               # solo phases: process `turn` runs, the other waits
        barrier.wait()
        if turn == idx:
            alone = timed()
        barrier.wait()
    barrier.wait()
    together = timed()                 # both at once
    q.put((idx, model, alone, together))


def measure_pair(a, b, steps, warmup):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    barrier, q = ctx.Barrier(2), ctx.SimpleQueue()
    ps = [ctx.Process(target=_proc, args=(i, m, steps, warmup, barrier, q)) for i, m in enumerate((a, b))]
    for p in ps:
        p.start()
    res = [q.get() for _ in ps]
    for p in ps:
        p.join(timeout=60)
        if p.exitcode != 0:
            raise RuntimeError(f"measurement process exited with {p.exitcode}")
    return {m: (al, tog) for _, m, al, tog in res} if a != b else \
        {a: (sum(r[2] for r in res) / 2, sum(r[3] for r in res) / 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="resnet50,vgg16,transformer,gnmt")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--out", default="profiles/interference_mi355x.json")
    a = ap.parse_args()
    models = a.models.split(",")
    slowdown, raw = {}, {}
    for x, y in itertools.combinations_with_replacement(models, 2):
        r = measure_pair(x, y, a.steps, a.warmup)
        for victim, (alone, together) in r.items():
            nb = y if victim == x else x
            s = together / alone
            slowdown[f"{victim}|{nb}"] = round(s, 4)
            raw[f"{victim}|{nb}"] = {"alone_ms": round(alone * 1e3, 3), "together_ms": round(together * 1e3, 3)}
            print(f"{victim:12s} with {nb:12s}: {alone * 1e3:8.2f} ms alone, {together * 1e3:8.2f} ms "
                  f"co-located -> slowdown {s:.3f}", flush=True)
    out = {"device": "MI355X (one GPU time-shared by two HIP processes)", "steps": a.steps,
           "slowdown": slowdown, "raw": raw}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
