"""Grouped weight-gradient GEMM on the Transformer-base problem set: one
grouped launch (csrc/kernels/gemm_grouped.hip) vs the per-layer gemm()
route, TF/s from HIP events (rocprof-friendly fixed repeat count).

    python tools/bench_grouped.py [--reps 20] [--tile 128|256] [--only grouped|single]
"""
from __future__ import annotations

import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def transformer_problems(tokens=4096, d=512, ffn=2048, layers=6, vocab=32000):
    """(M, N, has_bias) of every Linear weight gradient of one Transformer-base
    step (models/transformer.py), M = out features, N = in features."""
    enc = [(3 * d, d, 1), (d, d, 1), (ffn, d, 1), (d, ffn, 1)]
    dec = [(3 * d, d, 1), (d, d, 1), (d, d, 1), (d, d, 1), (ffn, d, 1), (d, ffn, 1)]
    probs = enc * layers + dec * layers + [(layers * 2 * d, d, 1), (vocab, d, 0)]
    return [(m, n, tokens, b) for m, n, b in probs]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tile", type=int, default=128)
    ap.add_argument("--only", default="", help="grouped | single (default both)")
    a = ap.parse_args()
    from tiresias_amd.ops import _lib

    _lib.load(required=True)
    T = torch.ops.tam
    T.gemm_lib_policy(0)
    T.gemm_grouped_tile(a.tile)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    probs = transformer_problems()
    dys = [torch.randn(K, M, device=dev).to(torch.bfloat16) for M, N, K, _ in probs]
    xs = [torch.randn(K, N, device=dev).to(torch.bfloat16) for M, N, K, _ in probs]
    dws = [torch.zeros(M, N, device=dev) for M, N, K, _ in probs]
    dbs = [torch.zeros(M, device=dev) if b else torch.empty(0, device=dev) for M, N, K, b in probs]
    flop = sum(2.0 * M * N * K for M, N, K, _ in probs)
    out = {"problems": len(probs), "gflop": flop / 1e9, "tile": a.tile}

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    if a.only in ("", "grouped"):
        ms = timed(lambda: T.gemm_wgrad_grouped(dys, xs, dws, dbs))
        out["grouped_ms"] = ms
        out["grouped_tflops"] = flop / ms / 1e9

    def single():
        for dy, x, dw, db in zip(dys, xs, dws, dbs):
            T.gemm(dy, False, x, False, dw, 1, None, False, None, 1.0, True, db if db.numel() else None)

    if a.only in ("", "single"):
        ms = timed(single)
        out["single_ms"] = ms
        out["single_tflops"] = flop / ms / 1e9
    print(json.dumps(out))


if __name__ == "__main__":
    main()
