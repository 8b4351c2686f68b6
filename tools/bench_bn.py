"""BatchNorm kernels on ResNet-50's layer shapes (bs 64 default): per-shape
time and achieved HBM bandwidth of the forward apply (statistics already
accumulated by the producing conv, as in the model), the backward
reduction and the backward apply, in the variants the model runs (relu with
the 1-bit mask, residual add + relu, plain). HIP-event timing, fixed repeat
count (rocprof-friendly).

    python tools/bench_bn.py [--batch 64] [--reps 20] [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def resnet50_bn_shapes(batch=64):
    """(name, M, C, kind): kind relu_mask (bn1/bn2: ReLU, backward mask in
    the consumer conv), relu_bits (stem: ReLU with 1-bit mask), res (bn3:
    residual add + ReLU), plain (downsample BN)."""
    out = [("stem", batch * 112 * 112, 64, "relu_bits")]
    H, cin = 56, 64
    for si, (n, w) in enumerate(zip((3, 4, 6, 3), (64, 128, 256, 512))):
        for bi in range(n):
            s = 2 if bi == 0 and si > 0 else 1
            Ho = H // s
            out.append((f"s{si}b{bi}.bn1", batch * H * H, w, "relu_mask"))
            out.append((f"s{si}b{bi}.bn2", batch * Ho * Ho, w, "relu_mask"))
            out.append((f"s{si}b{bi}.bn3", batch * Ho * Ho, 4 * w, "res"))
            if bi == 0:
                out.append((f"s{si}b{bi}.dbn", batch * Ho * Ho, 4 * w, "plain"))
            H = Ho
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from tiresias_amd.ops import _lib

    _lib.load(required=True)
    T = torch.ops.tam
    dev = torch.device("cuda", 0)
    BF = torch.bfloat16
    rows = []
    seen = {}
    for name, M, C, kind in resnet50_bn_shapes(a.batch):
        key = (M, C, kind)
        if key in seen:
            rows.append(dict(seen[key], name=name))
            continue
        x = torch.randn(M, C, device=dev).to(BF)
        res = torch.randn(M, C, device=dev).to(BF) if kind == "res" else None
        y = torch.empty_like(x)
        g = torch.ones(C, device=dev)
        b = torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        mean, rstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
        sums = torch.zeros(16 * 2 * C, dtype=torch.float64, device=dev)
        relu = kind != "plain"
        bits = kind in ("relu_bits", "res")
        ymask = torch.empty(M * C // 8, dtype=torch.uint8, device=dev) if bits else None
        # statistics as the producing conv leaves them (one full pass)
        T.bn_forward(x, res, y, g, b, rm, rv, mean, rstd, 1e-5, 0.1, relu, sums, False, ymask)
        dy = torch.randn(M, C, device=dev).to(BF)
        add = torch.randn(M, C, device=dev).to(BF) if kind == "res" else None
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if kind == "res" else None
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        bws = torch.zeros_like(sums)

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
            return e0.elapsed_time(e1) / a.reps * 1e3      # us

        fwd = timed(lambda: T.bn_forward(x, res, y, g, b, rm, rv, mean, rstd, 1e-5, 0.1, relu, sums, True,
                                         ymask))
        # backward as the model runs it: bn1 / bn2 get the consumer-masked
        # gradient (relu handled there), bn3 the residual addend + bit mask
        if kind == "relu_mask":
            bwd = timed(lambda: (T.bn_backward(dy, None, x, mean, rstd, g, dx, None, dg, db, False,
                                                            None, bws, False, None)))
        elif kind == "res":
            bwd = timed(lambda: (T.bn_backward(dy, None, x, mean, rstd, g, dx, dres, dg, db, True,
                                                            add, bws, False, ymask)))
        elif kind == "relu_bits":
            bwd = timed(lambda: (T.bn_backward(dy, None, x, mean, rstd, g, dx, None, dg, db, True,
                                                            None, bws, False, ymask)))
        else:
            bwd = timed(lambda: (T.bn_backward(dy, None, x, mean, rstd, g, dx, None, dg, db, False,
                                                            None, bws, False, None)))
        e = M * C * 2
        fwd_bytes = e * (3 if kind == "res" else 2) + (M * C // 8 if bits else 0)
        # reduce: dy, x (+ addend, mask, dres write); apply: dy(or dres), x, dx write
        bwd_bytes = {"relu_mask": 2 * e + 3 * e, "plain": 2 * e + 3 * e,
                     "relu_bits": 2 * e + 3 * e + 2 * M * C // 8,
                     "res": 3 * e + M * C // 8 + e + 3 * e}[kind]
        r = dict(name=name, M=M, C=C, kind=kind, fwd_us=round(fwd, 2), bwd_us=round(bwd, 2),
                 fwd_tbs=round(fwd_bytes / fwd / 1e6, 2), bwd_tbs=round(bwd_bytes / bwd / 1e6, 2))
        seen[key] = r
        rows.append(r)
        print(json.dumps(r), flush=True)
    tot_f = sum(r["fwd_us"] for r in rows)
    tot_b = sum(r["bwd_us"] for r in rows)
    summ = {"layers": len(rows), "fwd_total_us": round(tot_f, 1), "bwd_total_us": round(tot_b, 1)}
    print(json.dumps(summ))
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"summary": summ, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
