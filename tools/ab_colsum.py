"""A/B of the column-sum (bias gradient) paths on MI355X: partial rows + a
column-reduce launch (policy 1) vs one launch of <= 64 row blocks adding into
the output with fp32 atomics (policy 2). Each variant runs as a captured
hipGraph of 20 back-to-back calls (launch boundaries included, as in a
training step's graph); interleaved rounds, best of each.

  python tools/ab_colsum.py --out gpurun_out/ab_colsum.json
"""
from __future__ import annotations

import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

SHAPES = [(4096, 512), (4096, 2048), (4096, 1536), (3200, 4096), (3200, 32000), (64, 1000),
          (4096, 32000), (32 * 224 * 224, 64), (32 * 56 * 56, 256)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    _lib.load(required=True)
    T = torch.ops.tam
    dev = torch.device("cuda", 0)
    rows = []
    for R, C in SHAPES:
        x = torch.randn(R, C, device=dev).to(torch.bfloat16)
        ref = x.double().sum(0)
        best = {}
        for _ in range(a.rounds):
            for pol in (1, 2):
                T.colsum_policy(pol)
                out = torch.zeros(C, device=dev)
                T.colsum(x, out)
                torch.cuda.synchronize()
                err = float((out.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-9))
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    with torch.cuda.graph(g, stream=s):
                        for _ in range(20):
                            T.colsum(x, out)
                torch.cuda.synchronize()
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    g.replay()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / 200
                if pol not in best or us < best[pol][0]:
                    best[pol] = (us, err)
        T.colsum_policy(0)
        row = {"R": R, "C": C, "partial_us": round(best[1][0], 2), "atomic_us": round(best[2][0], 2),
               "err_partial": best[1][1], "err_atomic": best[2][1]}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
