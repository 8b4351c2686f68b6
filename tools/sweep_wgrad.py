"""Tile / split sweep of the LDS-DMA conv weight gradient (conv_dma.h) on every
ResNet-50 (bs 64) and VGG-16 (bs 32) wgrad shape: for each shape, time the
current heuristic, the register-staged igemm, and every forced (bm, bn,
splits) of the DMA kernel (tam.conv_wgrad_force). The split count sets the
fp32 atomic traffic (splits x |dW|, memory-side atomics at ~1.3 TB/s chip-wide)
against the MFMA work per block, so the best config is measured, not guessed.

  python tools/sweep_wgrad.py --out gpurun_out/sweep_wgrad.json
"""
from __future__ import annotations

import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

# (N, H, W, C, K, R, stride, pad, calls per step, model)
RN50 = [
    (64, 56, 56, 64, 64, 1, 1, 0, 1), (64, 56, 56, 256, 64, 1, 1, 0, 2), (64, 56, 56, 64, 64, 3, 1, 1, 3),
    (64, 56, 56, 64, 256, 1, 1, 0, 4),
    (64, 56, 56, 256, 128, 1, 1, 0, 1), (64, 56, 56, 128, 128, 3, 2, 1, 1), (64, 28, 28, 128, 512, 1, 1, 0, 4),
    (64, 56, 56, 256, 512, 1, 2, 0, 1), (64, 28, 28, 512, 128, 1, 1, 0, 3), (64, 28, 28, 128, 128, 3, 1, 1, 3),
    (64, 28, 28, 512, 256, 1, 1, 0, 1), (64, 28, 28, 256, 256, 3, 2, 1, 1), (64, 14, 14, 256, 1024, 1, 1, 0, 6),
    (64, 28, 28, 512, 1024, 1, 2, 0, 1), (64, 14, 14, 1024, 256, 1, 1, 0, 5), (64, 14, 14, 256, 256, 3, 1, 1, 5),
    (64, 14, 14, 1024, 512, 1, 1, 0, 1), (64, 14, 14, 512, 512, 3, 2, 1, 1), (64, 7, 7, 512, 2048, 1, 1, 0, 3),
    (64, 14, 14, 1024, 2048, 1, 2, 0, 1), (64, 7, 7, 2048, 512, 1, 1, 0, 2), (64, 7, 7, 512, 512, 3, 1, 1, 2),
]
VGG = [
    (32, 224, 224, 64, 64, 3, 1, 1, 1), (32, 112, 112, 64, 128, 3, 1, 1, 1), (32, 112, 112, 128, 128, 3, 1, 1, 1),
    (32, 56, 56, 128, 256, 3, 1, 1, 1), (32, 56, 56, 256, 256, 3, 1, 1, 2), (32, 28, 28, 256, 512, 3, 1, 1, 1),
    (32, 28, 28, 512, 512, 3, 1, 1, 2), (32, 14, 14, 512, 512, 3, 1, 1, 3),
]


def _time(fn, iters=10):
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
    return best * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="resnet50,vgg16")
    ap.add_argument("--out", default=None)
    ap.add_argument("--c64_ab", action="store_true",
                    help="3x3 stride-1 layers with C, K % 64 == 0 only: the patch-staged kernel (default grid; "
                         "64 / 256 blocks per slice) vs the tap-gather path, interleaved rounds, numerics")
    ap.add_argument("--atomic_ab", action="store_true",
                    help="only time the heuristic with atomics vs racy plain adds (prices the atomics)")
    ap.add_argument("--order_ab", action="store_true",
                    help="heuristic config, 3-D grid vs split-major flat XCD order (conv_wgrad_order), interleaved")
    ap.add_argument("--slab_ab", action="store_true",
                    help="heuristic config, fp32-atomic split epilogue vs slab partials + reduce "
                         "(conv_wgrad_slab_policy), interleaved, both store and accumulate modes")
    ap.add_argument("--slab", type=int, default=1, help="slab policy for the other modes")
    ap.add_argument("--min_hw", type=int, default=0, help="only shapes with H >= this")
    ap.add_argument("--no_c64", action="store_true",
                    help="patch-staged 64-channel kernel off (the path a side-stream wgrad takes)")
    ap.add_argument("--splits", default="1,2,4,8,16,32,64,128", help="forced split counts to sweep")
    a = ap.parse_args()
    _lib.load(required=True)
    T = torch.ops.tam
    T.conv_wgrad_slab_policy(a.slab)
    if a.no_c64:
        T.conv_wgrad_c64_policy(0)
    dev = torch.device("cuda", 0)
    shapes = [("resnet50",) + s for s in RN50] * ("resnet50" in a.models) + \
             [("vgg16",) + s for s in VGG] * ("vgg16" in a.models)
    out = []
    for model, N, H, W, C, K, R, st, pd, calls in shapes:
        if H < a.min_hw:
            continue
        P = (H + 2 * pd - R) // st + 1
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(N, P, P, K, device=dev).to(torch.bfloat16)
        dw = torch.zeros(K, R, R, C, device=dev)
        run = lambda: T.conv_wgrad(dy, x, dw, st, pd, 1, 1)  # noqa: E731
        T.conv_wgrad_force(0, 0, 0)
        dw.zero_(); run(); torch.cuda.synchronize(); ref = dw.clone()
        row = {"model": model, "shape": [N, H, W, C, K, R, st, pd], "calls": calls,
               "auto_us": round(_time(run), 2)}
        if a.c64_ab:
            if not (C % 64 == 0 and K % 64 == 0 and R == 3 and st == 1):
                continue
            best = {}
            for _ in range(2):
                for pol in (0, 1, 64, 256):
                    T.conv_wgrad_c64_policy(pol)
                    best[pol] = min(best.get(pol, 1e9), _time(run))
            T.conv_wgrad_c64_policy(0)
            dw.zero_(); run(); torch.cuda.synchronize(); r0 = dw.clone()
            T.conv_wgrad_c64_policy(1)
            dw.zero_(); run(); torch.cuda.synchronize()
            row.update({"gather_us": round(best[0], 2), "c64_us": round(best[1], 2), "c64_g64_us": round(best[64], 2),
                        "c64_g256_us": round(best[256], 2),
                        "rel_diff": float((dw - r0).norm() / r0.norm().clamp_min(1e-30))})
            out.append(row)
            print(json.dumps(row), flush=True)
            continue
        if a.slab_ab:
            best = {}
            run0 = lambda: T.conv_wgrad(dy, x, dw, st, pd, 1, 0)  # noqa: E731  (store mode)
            for _ in range(3):
                for o in (0, 1):
                    T.conv_wgrad_slab_policy(o)
                    best[o] = min(best.get(o, 1e9), _time(run))
                    best[o + 2] = min(best.get(o + 2, 1e9), _time(run0))
            T.conv_wgrad_slab_policy(0)
            dw.normal_(); run0(); torch.cuda.synchronize(); r0 = dw.clone()
            T.conv_wgrad_slab_policy(1)
            dw.normal_(); run0(); torch.cuda.synchronize()
            d0 = float((dw - r0).norm() / r0.norm().clamp_min(1e-30))
            dw.copy_(r0); run(); torch.cuda.synchronize()
            d1 = float((dw - 2 * r0).norm() / (2 * r0).norm().clamp_min(1e-30))
            T.conv_wgrad_slab_policy(a.slab)
            row.update({"atomic_us": round(best[0], 2), "slab_us": round(best[1], 2),
                        "atomic_store_us": round(best[2], 2), "slab_store_us": round(best[3], 2),
                        "rel_diff_store": d0, "rel_diff_acc": d1})
            out.append(row)
            print(f"{model:8s} {str(row['shape']):38s} x{calls} acc: atomic {best[0]:7.2f} slab {best[1]:7.2f} | "
                  f"store: atomic {best[2]:7.2f} slab {best[3]:7.2f} | diff {d0:.1e} {d1:.1e}", flush=True)
            continue
        if a.order_ab:
            best = {}
            for _ in range(3):
                for o in (0, 1):
                    T.conv_wgrad_order(o)
                    best[o] = min(best.get(o, 1e9), _time(run))
            T.conv_wgrad_order(0)
            dw.zero_(); run(); torch.cuda.synchronize(); r0 = dw.clone()
            T.conv_wgrad_order(1)
            dw.zero_(); run(); torch.cuda.synchronize()
            row.update({"grid3d_us": round(best[0], 2), "flat_us": round(best[1], 2),
                        "rel_diff": float((dw - r0).norm() / r0.norm().clamp_min(1e-30))})
            out.append(row)
            print(f"{model:8s} {str(row['shape']):38s} x{calls} 3d {row['grid3d_us']:7.2f} "
                  f"flat {row['flat_us']:7.2f} diff {row['rel_diff']:.1e}", flush=True)
            continue
        if a.atomic_ab:
            T.conv_wgrad_force(0, 0, 0, 1)
            row["noatomic_us"] = round(_time(run), 2)
            T.conv_wgrad_force(0, 0, 0, 0)
            out.append(row)
            print(f"{model:8s} {str(row['shape']):38s} x{calls} auto {row['auto_us']:7.2f} "
                  f"no-atomic {row['noatomic_us']:7.2f}", flush=True)
            continue
        T.conv_dma_policy(0)
        row["igemm_us"] = round(_time(run), 2)
        T.conv_dma_policy(1)
        nsteps = (N * P * P + 63) // 64
        cfgs = {}
        for bm, bn in ((256, 128), (256, 64), (128, 128), (128, 64), (64, 64)):
            if K % bm or C % bn:
                continue
            for sp in [int(v) for v in a.splits.split(",")]:
                if sp > max(1, nsteps // 2):
                    continue
                T.conv_wgrad_force(bm, bn, sp)
                dw.zero_(); run(); torch.cuda.synchronize()
                err = float((dw - ref).norm() / ref.norm().clamp_min(1e-30))
                if err > 1e-3:
                    cfgs[f"{bm}x{bn}/{sp}"] = {"us": None, "err": err}
                    continue
                cfgs[f"{bm}x{bn}/{sp}"] = {"us": round(_time(run), 2)}
        T.conv_wgrad_force(0, 0, 0)
        ok = {k: v["us"] for k, v in cfgs.items() if v.get("us") is not None}
        best = min(ok, key=ok.get) if ok else None
        row["cfgs"] = cfgs
        row["best"] = best
        row["best_us"] = ok.get(best)
        out.append(row)
        print(f"{model:8s} {str(row['shape']):38s} x{calls} auto {row['auto_us']:7.2f} igemm {row['igemm_us']:7.2f} "
              f"best {best} {row['best_us']}", flush=True)
        del x, dy, dw, ref
    tot = {k: sum(r[k] * r["calls"] for r in out if r.get(k))
           for k in ("auto_us", "igemm_us", "best_us", "noatomic_us", "grid3d_us", "flat_us",
                     "atomic_us", "slab_us", "atomic_store_us", "slab_store_us")}
    print("per-step totals (us):", {k: round(v, 1) for k, v in tot.items()})
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"rows": out, "totals_us": tot}, f, indent=1)


if __name__ == "__main__":
    main()
