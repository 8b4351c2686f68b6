"""The 64x128 gemm8p tile (K-major A) vs the tiles it competes with on the
shapes it exists for: the Transformer's N = 512 projections and their
data gradients (4096 x 512 x K: 256 tiles of 64x128 = one per CU, where the
128^2 tile makes 128 blocks and the 256^2 tile 32). Per shape: the
register-staged igemm (the route these shapes took in round 6's library-off
table), gemm8p 128^2 and 64x128 forced, unsplit and with slab split-K.
Random uniform bf16 operands (guide §5.4 rule 25). One JSON line per shape.

    python tools/bench_gemm_tile64.py [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

BF = torch.bfloat16
# (M, N, K, b K-major) -- A is K-major in all of them (activations x W^T,
# dY x W); the wide-N K=512 shapes are there to see where the tile stops paying
SHAPES = [(4096, 512, 512, True), (4096, 512, 512, False), (4096, 512, 1536, False),
          (4096, 512, 2048, True), (4096, 512, 2048, False), (4096, 1536, 512, True),
          (4096, 2048, 512, True), (4096, 2048, 512, False), (3200, 1024, 1024, True),
          (3200, 1024, 1024, False), (3200, 2048, 1024, True), (3200, 1024, 2048, False),
          (3200, 1024, 4096, True)]


def timeit(fn, iters=20):
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


# ResNet-50's pointwise convs at batch 64 (M = N x H x W output pixels,
# short K): forward x W^T (KK) and data gradient dY W (KN), --resnet
RESNET = [(200704, 256, 64, True), (200704, 64, 256, True), (200704, 64, 64, True),
          (50176, 512, 128, True), (50176, 128, 512, True), (12544, 1024, 256, True),
          (12544, 256, 1024, True), (3136, 2048, 512, True), (3136, 512, 2048, True),
          (200704, 64, 256, False), (200704, 256, 64, False), (50176, 128, 512, False),
          (12544, 256, 1024, False)]


def main():
    global SHAPES
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--resnet", action="store_true", help="ResNet-50 pointwise conv shapes")
    a = ap.parse_args()
    if a.resnet:
        SHAPES = RESNET
    T = _lib.ops()
    T.gemm_lib_policy(0)
    T.gemm_dma_policy(0, -1)      # no per-shape route timing: each forced config runs as asked
    dev = torch.device("cuda", 0)
    rows = []
    for M, N, K, bk in SHAPES:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(BF)
        B = (torch.rand(K, N, device=dev) * 2 - 1).to(BF)
        b_ = B.t().contiguous() if bk else B
        c = torch.empty(M, N, device=dev, dtype=BF)
        ref = A.float() @ B.float()
        fl = 2.0 * M * N * K
        r = {"shape": f"{M}x{N}x{K} K{'K' if bk else 'N'}"}
        for name, mode, tile, sp in (("igemm", 0, 0, 0), ("p8_128", 2, 128, 0), ("p8_64", 2, 64, 0), ("p8_65", 2, 65, 0), ("p8_129", 2, 129, 0),
                                     ("p8_256", 2, 256, 0), ("p8_128_slab", 3, 128, 0), ("p8_64_slab2", 3, 64, 2)):
            if (sp and K // 64 < 8 * sp) or (mode == 3 and K < 1024):
                continue
            T.gemm8p_policy(mode, tile)
            T.gemm8p_slab_force(sp)
            c.zero_()
            T.gemm(A, True, b_, bk, c, 0, None, False, None, 1.0, False)
            torch.cuda.synchronize()
            err = ((c.float() - ref).norm() / ref.norm()).item()
            assert err < 1e-2, (r["shape"], name, err)
            ms = timeit(lambda: T.gemm(A, True, b_, bk, c, 0, None, False, None, 1.0, False))
            r[name + "_us"] = round(ms * 1e3, 2)
            r[name + "_tflops"] = round(fl / ms / 1e9, 1)
        T.gemm8p_slab_force(0)
        T.gemm8p_policy(1, 0)
        Be = b_.t() if bk else b_
        ms = timeit(lambda: torch.mm(A, Be, out=c))
        r["hipblaslt_us"] = round(ms * 1e3, 2)
        r["min_bytes_tbps_igemm"] = round((M * K + N * K + M * N) * 2 / (r["igemm_us"] * 1e-6) / 1e12, 2)
        rows.append(r)
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
