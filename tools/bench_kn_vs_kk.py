"""Is a K-major copy of a weight worth its transpose? dX = dY . W with W
[N_out... ] stored N-major (the KN layout) against the same product with W
re-laid K-major (KK), both through the measured routing (library off), plus
the batched weight re-lay that would produce the K-major copies
(conv_weight_t_batch, as 1x1 "conv" weights). GNMT's shapes: the LSTM input
gradients (3200 x I x 4H) and the classifier's (3200 x 2H x V).

    python tools/bench_kn_vs_kk.py [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

BF = torch.bfloat16
SHAPES = [(3200, 1024, 4096), (3200, 2048, 4096), (3200, 2048, 32000)]


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    best = 1e9
    for _ in range(5):
        ev[0].record()
        for _ in range(iters):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        best = min(best, ev[0].elapsed_time(ev[1]) / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    T = _lib.ops()
    T.gemm_lib_policy(0)
    dev = torch.device("cuda", 0)
    rows = []
    for M, N, K in SHAPES:
        dy = (torch.rand(M, K, device=dev) * 2 - 1).to(BF)          # [M][K] K-major A
        W = (torch.rand(K, N, device=dev) * 2 - 1).to(BF)           # [K][N]: the stored weight (N-major B)
        Wt = torch.empty(N, K, device=dev, dtype=BF)
        c = torch.empty(M, N, device=dev, dtype=BF)
        T.conv_weight_t_batch([W.view(K, 1, 1, N)], [Wt])
        torch.cuda.synchronize()
        assert torch.equal(Wt, W.t().contiguous())
        kn = timeit(lambda: T.gemm(dy, True, W, False, c, 0, None, False, None, 1.0, False))
        ref = c.clone()
        kk = timeit(lambda: T.gemm(dy, True, Wt, True, c, 0, None, False, None, 1.0, False))
        assert ((c.float() - ref.float()).norm() / ref.float().norm()).item() < 1e-2
        tr = timeit(lambda: T.conv_weight_t_batch([W.view(K, 1, 1, N)], [Wt]))
        r = {"shape": f"{M}x{N}x{K}", "kn_us": round(kn * 1e3, 2), "kk_us": round(kk * 1e3, 2),
             "transpose_us": round(tr * 1e3, 2), "weight_mb": round(W.numel() * 2 / 2**20, 1),
             "transpose_tbps": round(2 * W.numel() * 2 / tr / 1e9, 2)}
        print(json.dumps(r), flush=True)
        rows.append(r)
    print(T.gemm_routes(), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
