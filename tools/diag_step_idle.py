"""Where does a graph-replayed training step spend its wall time?

For each model: steady-state ms/step, the host time spent inside
``Trainer.step()`` (graph replay submission + eager optimizer launch), and
the GPU time of the replay alone and of the optimizer alone (hipEvents on the
stream). If GPU time << wall time, the step is host-submission bound.

  python tools/diag_step_idle.py --models gnmt,resnet50
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.executor.trainer import Trainer  # noqa: E402


def diag(model: str, steps: int) -> dict:
    dev = torch.device("cuda", 0)
    t = Trainer(model, dev, use_graph=True)
    for _ in range(4):
        t.step()
    torch.cuda.synchronize()
    # wall per step, back to back
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(steps):
        h0 = time.perf_counter()
        t.step()
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    # GPU time of replay vs optimizer, each bracketed by events (synchronised
    # per step so submission cannot hide behind execution)
    s = torch.cuda.current_stream(dev)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    g_ms = o_ms = sub_ms = 0.0
    for _ in range(steps):
        torch.cuda.synchronize()
        e[0].record(s)
        h0 = time.perf_counter()
        t._graph.replay()
        sub_ms += (time.perf_counter() - h0) * 1e3
        e[1].record(s)
        t._opt_step()
        e[2].record(s)
        torch.cuda.synchronize()
        g_ms += e[0].elapsed_time(e[1])
        o_ms += e[1].elapsed_time(e[2])
    return dict(model=model, wall_ms=wall * 1e3, host_ms_in_step=host / steps * 1e3,
                replay_submit_ms=sub_ms / steps, graph_gpu_ms=g_ms / steps, opt_gpu_ms=o_ms / steps)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="gnmt,resnet50,transformer,vgg16")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    from tiresias_amd.ops import _lib

    _lib.load(required=True)
    for m in a.models.split(","):
        print(json.dumps(diag(m, a.steps)), flush=True)


if __name__ == "__main__":
    main()
