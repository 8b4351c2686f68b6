"""Stream-K schedule of the 256^2 gemm8p kernel (csrc/kernels/gemm8p_sk.hip)
vs the uniform slab split-K configurations and hipBLASLt on the GNMT
few-tile / long-K shapes. HIP-event timing, best of 5 bursts of 10 calls;
run under rocprofv3 --kernel-trace --stats to split main loop vs fixup.

    python tools/bench_streamk.py [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

BF = torch.bfloat16
SHAPES = [(3200, 2048, 32000, "KN"), (3200, 2048, 4096, "KN"), (3200, 1024, 4096, "KN"),
          (4096, 1024, 3200, "MN"), (2048, 1024, 3200, "MN"), (4096, 4096, 4096, "KK")]


def timeit(fn, iters=10):
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
    for M, N, K, lay in SHAPES:
        ak, bk = lay[0] == "K", lay[1] == "K"
        f32 = lay == "MN"                 # the weight-gradient shapes accumulate fp32
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(BF)
        B = (torch.rand(K, N, device=dev) * 2 - 1).to(BF)
        a_ = A if ak else A.t().contiguous()
        b_ = B.t().contiguous() if bk else B
        c = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else BF)
        mode = 1 if f32 else 0
        fn = lambda: T.gemm(a_, ak, b_, bk, c, mode, None, False, None, 1.0, True)  # noqa: E731
        r = {"shape": f"{M}x{N}x{K} {lay}", "f32_acc": f32}
        T.gemm8p_policy(3, 0)
        T.gemm8p_sk_force(1)
        r["streamk_us"] = round(timeit(fn), 2)
        T.gemm8p_sk_force(0)
        for tile in (256, 128):
            for sp in (1, 2, 3, 4, 5, 7, 8):
                if K // 64 // sp < 8:
                    continue
                T.gemm8p_policy(3, tile)
                T.gemm8p_slab_force(sp)
                r[f"p8_{tile}_sp{sp}_us"] = round(timeit(fn), 2)
        T.gemm8p_slab_force(0)
        T.gemm8p_policy(1, 0)
        Ae, Be = A, B
        if f32:
            # store-only fp32 (what bench_gemm_routes times) and accumulate into C (what ours does)
            r["lib_us"] = round(timeit(lambda: torch.mm(Ae, Be, out_dtype=torch.float32)), 2)
            try:
                r["lib_acc_us"] = round(timeit(lambda: torch.addmm(c, Ae, Be, out_dtype=torch.float32, out=c)), 2)
            except Exception as e:      # overload not exposed in this build
                r["lib_acc_us"] = str(e)[:80]
        else:
            r["lib_us"] = round(timeit(lambda: torch.mm(Ae, Be, out=c)), 2)
        best = min((v, k) for k, v in r.items() if k.endswith("_us") and not k.startswith("lib"))
        r["best"], r["best_us"] = best[1], best[0]
        r["tflops_best"] = round(2.0 * M * N * K / best[0] / 1e6, 1)
        print(json.dumps(r), flush=True)
        rows.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
