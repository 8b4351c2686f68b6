"""Per-model training throughput on one MI355X through the tiresias_amd
kernels (samples/s and ms/step), with a rocprof-friendly fixed step count.
These per-iteration times are also what the cluster simulator's job model
uses (``--throughput_table``)."""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.executor.trainer import Trainer  # noqa: E402


def bench(model, batch=None, steps=10, warmup=3, graph=False):
    dev = torch.device("cuda", 0)
    t = Trainer(model, dev, batch=batch, use_graph=graph)
    for _ in range(warmup):
        t.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        t.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return dict(model=model, batch=t.batch, graph=graph, ms_per_step=dt * 1e3,
                samples_per_s=t.samples_per_step() / dt, loss=float(t.last_loss),
                params=t.arena.numel, state_mb=t.state_bytes() / 2 ** 20)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="resnet50,vgg16,transformer,gnmt")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = []
    for m in a.models.split(","):
        r = bench(m, steps=a.steps, warmup=a.warmup, graph=a.graph)
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
