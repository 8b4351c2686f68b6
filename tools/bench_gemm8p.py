"""gemm8p (256^2 all-layout LDS-DMA GEMM) vs the previous kernels vs
hipBLASLt, on the model zoo's big plain GEMMs and square sizes. Random
uniform bf16 operands (guide §5.4 rule 25). One JSON list to --out."""
from __future__ import annotations

import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

BF = torch.bfloat16
SHAPES = [(4096, 4096, 4096, True, True), (8192, 8192, 8192, True, True),
          (4096, 4096, 4096, True, False), (4096, 4096, 4096, False, True), (4096, 4096, 4096, False, False),
          # GNMT / Transformer vocab projections and gradients (profiles/gnmt_branches_r1/off.log)
          (3200, 32000, 2048, True, True), (3200, 2048, 32000, True, False), (32000, 2048, 3200, False, False),
          (3200, 2048, 4096, True, False), (3200, 1024, 4096, True, False), (4096, 2048, 3200, False, False),
          (4096, 32000, 512, True, True), (4096, 512, 32000, True, False), (32000, 512, 4096, False, False),
          (3200, 4096, 1024, True, True), (2048, 1024, 3200, False, False)]


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    best = 1e9
    for _ in range(3):
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
    ap.add_argument("--ablate", action="store_true", help="4096^3 KK: no-DMA / no-LDS-read ceilings")
    a = ap.parse_args()
    T = _lib.ops()
    T.gemm_lib_policy(0)
    dev = torch.device("cuda", 0)
    rows = []
    if a.ablate:
        M = N = K = 4096
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(BF)
        B = (torch.rand(N, K, device=dev) * 2 - 1).to(BF)
        c = torch.empty(M, N, device=dev, dtype=BF)
        for name, tile in (("p8_256", 256), ("p8_128", 128)):
            T.gemm8p_policy(2, tile)
            ms = timeit(lambda: T.gemm(A, True, B, True, c, 0, None, False, None, 1.0, False))
            print(json.dumps({"ablation": name, "tflops": round(2.0 * M * N * K / ms / 1e9, 1)}), flush=True)
        T.gemm8p_policy(1, 0)
        return
    for (M, N, K, ak, bk) in SHAPES:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(BF)
        B = (torch.rand(K, N, device=dev) * 2 - 1).to(BF)
        a_ = A if ak else A.t().contiguous()
        b_ = B.t().contiguous() if bk else B
        c = torch.empty(M, N, device=dev, dtype=BF)
        fl = 2.0 * M * N * K
        res = {"shape": f"{M}x{N}x{K} {'K' if ak else 'M'}{'K' if bk else 'N'}"}
        for name, mode, stg in (("p8_256", 2, 256), ("p8_128", 2, 128), ("p8_slab_auto", 3, 0),
                                ("legacy", 0, 0)):
            T.gemm8p_policy(mode, stg)
            ms = timeit(lambda: T.gemm(a_, ak, b_, bk, c, 0, None, False, None, 1.0, False))
            res[name + "_tflops"] = round(fl / ms / 1e9, 1)
        cf = torch.zeros(M, N, device=dev)
        for name, mode, stg in (("p8_f32acc_auto", 2, 0), ("p8slab_f32acc_auto", 3, 0)):
            T.gemm8p_policy(mode, stg)
            ms = timeit(lambda: T.gemm(a_, ak, b_, bk, cf, 1, None, False, None, 1.0, False))
            res[name + "_tflops"] = round(fl / ms / 1e9, 1)
        T.gemm8p_policy(1, 0)
        Ae = a_ if ak else a_.t()          # same memory layouts as our kernel sees
        Be = b_.t() if bk else b_

        def lib():
            torch.mm(Ae, Be, out=c)
        ms = timeit(lib)
        res["hipblaslt_tflops"] = round(fl / ms / 1e9, 1)
        rows.append(res)
        print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
