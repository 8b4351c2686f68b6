"""Skinny-M weight-streaming GEMM (csrc/kernels/gemm_skinny.hip) on the VGG
classifier's batch-32 shapes: K-slice count x LDS ring depth sweep, the
heuristic's pick, hipBLASLt (torch.mm) on the same layout, and the achieved
weight-stream bandwidth. HIP-event timing, best of 5 bursts of 20 calls.

    python tools/bench_skinny.py [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

BF = torch.bfloat16
# (M, N, K, W K-major?): fc0 fwd / dgrad, fc1 fwd / dgrad, fc2 fwd / dgrad
SHAPES = [(32, 4096, 25088, True), (32, 25088, 4096, False), (32, 4096, 4096, True), (32, 4096, 4096, False),
          (32, 1000, 4096, True), (32, 4096, 1000, False)]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return best * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    T = _lib.ops()
    T.gemm_lib_policy(0)
    dev = torch.device("cuda", 0)
    rows = []
    for M, N, K, bk in SHAPES:
        x = torch.randn(M, K, device=dev).to(BF)
        W = (torch.randn(N, K, device=dev) / 8).to(BF)
        b = W if bk else W.t().contiguous()
        y = torch.empty(M, N, device=dev, dtype=BF)
        wbytes = N * K * 2
        res = {"shape": f"{M}x{N}x{K} {'KK' if bk else 'KN'}"}
        for nst in (3, 4):
            for sp in (0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32):
                if sp and sp > K // 64 // 2:
                    continue
                T.gemm_skinny_policy(1, sp, nst)
                us = timeit(lambda: T.gemm(x, True, b, bk, y, 0, None, False, None, 1.0, False))
                res[f"nst{nst}_sp{sp or 'auto'}"] = round(us, 2)
        T.gemm_skinny_policy(1, 0, 3)
        Be = b.t() if bk else b
        res["lib_us"] = round(timeit(lambda: torch.mm(x, Be, out=y)), 2)
        best = min((v, k) for k, v in res.items() if k.startswith("nst"))
        res["best"] = best[1]
        res["best_us"] = best[0]
        res["auto_us"] = res["nst3_spauto"]
        res["auto_tbs"] = round(wbytes / res["auto_us"] / 1e6, 2)
        res["best_tbs"] = round(wbytes / best[0] / 1e6, 2)
        print(json.dumps(res), flush=True)
        rows.append(res)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
