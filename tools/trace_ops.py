"""Per-layer kernel budget of one eager training step: every call a model makes
into the HIP op library (conv fwd/dgrad/wgrad, BN passes, GEMMs, pools, ...)
is recorded with its argument shapes, then each distinct call is replayed in
isolation (cloned arguments, hipEvent timing, best of 3 x `iters`) and the
table prints per-step cost = time x calls, largest first. Finds the layers
worth fusing or re-tiling without guessing from kernel-name aggregates.

  python tools/trace_ops.py --model resnet50 --top 60 --out gpurun_out/ops_rn50.json
"""
from __future__ import annotations

import argparse
import collections
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.executor.trainer import Trainer  # noqa: E402
from tiresias_amd.ops import _lib  # noqa: E402


def _sig(v):
    if isinstance(v, torch.Tensor):
        return "x".join(map(str, v.shape)) + ":" + str(v.dtype).replace("torch.", "")
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(_sig(x) for x in v) + "]"
    if isinstance(v, float):
        return f"{v:g}"
    return str(v)


def _clone(v):
    if isinstance(v, torch.Tensor):
        return v.detach().clone()
    if isinstance(v, (list, tuple)):
        return type(v)(_clone(x) for x in v)
    return v


class _Recorder:
    SKIP = {"gemm_routes", "gemm_routes_load", "lstm_persist_timeouts"}

    def __init__(self, real):
        self.real = real
        self.calls = collections.Counter()
        self.example = {}
        self.order = []

    def __getattr__(self, name):
        fn = getattr(self.real, name)
        if name in self.SKIP or not callable(fn):
            return fn

        def wrapped(*args):
            key = name + "(" + ", ".join(_sig(a) for a in args) + ")"
            self.calls[key] += 1
            if key not in self.example:
                self.example[key] = (name, [_clone(a) for a in args])
                self.order.append(key)
            return fn(*args)
        return wrapped


def _time(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return best * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--top", type=int, default=50)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    _lib.load(required=True)
    T = torch.ops.tam
    dev = torch.device("cuda", 0)
    t = Trainer(a.model, dev, use_graph=False)
    t.step()                       # warm: routes tuned, buffers allocated
    torch.cuda.synchronize()
    rec = _Recorder(T)
    orig = _lib.ops
    _lib.ops = lambda: rec
    try:
        t.step()
        torch.cuda.synchronize()
    finally:
        _lib.ops = orig
    rows = []
    for key in rec.order:
        name, args = rec.example[key]
        fn = getattr(T, name)
        us = _time(lambda: fn(*args), a.iters)
        rows.append({"op": key, "calls": rec.calls[key], "us": round(us, 2),
                     "us_per_step": round(us * rec.calls[key], 2)})
        del args
    torch.cuda.empty_cache()
    rows.sort(key=lambda r: -r["us_per_step"])
    total = sum(r["us_per_step"] for r in rows)
    by_op = collections.Counter()
    for r in rows:
        by_op[r["op"].split("(")[0]] += r["us_per_step"]
    print(f"# {a.model}: {len(rows)} distinct calls, {sum(rec.calls.values())} calls/step, "
          f"sum of isolated times {total / 1e3:.3f} ms")
    for k, v in by_op.most_common():
        print(f"#   {k:24s} {v / 1e3:7.3f} ms  {100 * v / total:5.1f} %")
    for r in rows[:a.top]:
        print(f"{r['us_per_step']:9.1f} us/step  {r['calls']:3d} x {r['us']:8.2f}  {r['op'][:200]}")
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"model": a.model, "total_us": total, "by_op_us": dict(by_op), "rows": rows}, f,
                      indent=1)


if __name__ == "__main__":
    main()
