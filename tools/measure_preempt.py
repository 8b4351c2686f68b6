"""Measure what a preemption costs a job on the live runtime (one GPU):

* ``build``    -- a fresh Trainer (allocation + init) until its first
                  graph step is done (2 eager warm-up steps + capture);
* ``pool``     -- a warm-pool reuse (``Trainer.reset``) + one step;
* ``step``     -- one steady-state (graph-replay) step;
* ``spill``    -- host time of ``offload`` (async) and device D2H time;
* ``resume``   -- ``restore`` + the first step after it, device-synchronised
                  (H2D + graph re-capture when the addresses moved).

Prints one JSON line per model.
"""
from __future__ import annotations

import argparse
import json
import time

import torch

from tiresias_amd.executor.trainer import Trainer


def _t(fn, dev):
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="transformer,gnmt")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from tiresias_amd.ops import _lib

    _lib.load(required=True)
    eng = torch.classes.tam.CkptEngine(0, 1 << 30)
    for m in a.models.split(","):
        box = {}
        build = _t(lambda: box.setdefault("t", Trainer(m, dev, use_graph=True)).run(3), dev)
        t = box["t"]
        step = min(_t(lambda: t.step(), dev) for _ in range(5))
        pool = _t(lambda: (t.reset(1), t.step()), dev)
        t.run(3)
        spill_host, resume, d2h, h2d = [], [], [], []
        for _ in range(a.reps):
            torch.cuda.synchronize(dev)
            h = time.perf_counter()
            t.offload(eng)
            spill_host.append((time.perf_counter() - h) * 1e3)
            torch.cuda.synchronize(dev)
            resume.append(_t(lambda: (t.restore(), t.step()), dev))
            c = t.ckpt_poll()
            d2h.append(c["save_s"] * 1e3)
            h2d.append(c["restore_s"] * 1e3)
            t.run(2)
        print(json.dumps({"model": m, "state_gb": round(t.state_bytes() / 2 ** 30, 3),
                          "build_ms": round(build, 1), "step_ms": round(step, 2), "pool_ms": round(pool, 1),
                          "spill_host_ms": [round(x, 2) for x in spill_host],
                          "d2h_ms": [round(x, 1) for x in d2h], "h2d_ms": [round(x, 1) for x in h2d],
                          "resume_ms": [round(x, 1) for x in resume]}), flush=True)
        t.release()
        del t, box
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
