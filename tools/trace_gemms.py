"""Per-model GEMM budget: record every tam.gemm call one eager training step
of a model makes (shape, operand majorities, output dtype, epilogue, split),
then time each distinct call in isolation through each available path —
the shipped routing (our kernels) and hipBLASLt for reference — and
print the per-step cost of each shape x calls. Used to decide the plain-GEMM
routing policy from measurements instead of guesses.

  python tools/trace_gemms.py --models transformer,gnmt --out profiles/gemm_budget.json
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


class _Recorder:
    def __init__(self, real):
        self.real = real
        self.calls = collections.Counter()
        self.example = {}

    def __getattr__(self, name):
        return getattr(self.real, name)

    def gemm(self, a, ak, b, bk, c, mode, bias, relu, mask, alpha, allow_split, colsum=None):
        M, N = c.shape[-2] if c.dim() > 1 else 1, c.shape[-1]
        M = c.numel() // N
        K = a.shape[-1] if ak else a.shape[0]
        key = (M, N, K, ak, bk, str(c.dtype).replace("torch.", ""), int(mode), bias is not None,
               bool(relu), mask is not None, bool(allow_split))
        self.calls[key] += 1
        if key not in self.example:
            self.example[key] = (a.detach().clone(), b.detach().clone(), c.detach().clone(),
                                 None if bias is None else bias.detach().clone(),
                                 None if mask is None else mask.detach().clone())
        return self.real.gemm(a, ak, b, bk, c, mode, bias, relu, mask, alpha, allow_split, colsum)


def _time(fn, iters=20):
    for _ in range(3):
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
    ap.add_argument("--models", default="transformer,gnmt,resnet50,vgg16")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    _lib.load(required=True)
    T = torch.ops.tam
    dev = torch.device("cuda", 0)
    report = {}
    for m in a.models.split(","):
        rec = _Recorder(T)
        orig = _lib.ops
        _lib.ops = lambda: rec
        try:
            t = Trainer(m, dev, use_graph=False)
            t.step()
            torch.cuda.synchronize()
        finally:
            _lib.ops = orig
        rows = []
        for key, n in rec.calls.items():
            M, N, K, ak, bk, dt, mode, has_b, relu, has_m, split = key
            A, B, C, bias, mask = rec.example[key]
            res = {}
            # "route": the shipped routing (production default, library off);
            # "lib": hipBLASLt on the same layouts, for reference only
            for path, lib in {"route": 0, "lib": 1}.items():
                if path == "lib" and (relu or has_m):
                    continue
                T.gemm_lib_policy(lib)
                cc = C.clone()
                res[path] = _time(lambda: T.gemm(A, ak, B, bk, cc, mode, bias, relu, mask, 1.0, split))
            T.gemm_lib_policy(0)
            best = min(res, key=res.get)
            rows.append(dict(M=M, N=N, K=K, layout=("K" if ak else "M") + ("K" if bk else "N"),
                             out=dt, mode=mode, bias=has_b, relu=relu, mask=has_m, split=split,
                             calls=n, us=res, best=best, step_us={p: v * n for p, v in res.items()}))
        rows.sort(key=lambda r: -min(r["step_us"].values()))
        tot = {p: sum(r["step_us"].get(p, r["step_us"]["route"]) for r in rows) for p in ("route", "lib")}
        tot["best"] = sum(min(r["step_us"].values()) for r in rows)
        print(f"== {m}: per-step GEMM us by path {json.dumps({k: round(v) for k, v in tot.items()})}")
        for r in rows:
            print(f"  {r['M']:6d}x{r['N']:6d}x{r['K']:6d} {r['layout']} {r['out']:8s} mode{r['mode']} "
                  f"b{int(r['bias'])} r{int(r['relu'])} m{int(r['mask'])} s{int(r['split'])} x{r['calls']:4d} "
                  + " ".join(f"{p}={v:7.1f}" for p, v in r["us"].items()) + f"  best={r['best']}")
        report[m] = dict(total_us=tot, shapes=rows)
    if a.out:
        json.dump(report, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
