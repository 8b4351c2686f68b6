"""TF/s of the production GEMM routing (gemm8p, tile forced or
auto) on square and model shapes, one JSON line per shape; run once per
library build (TAM_LIB_PATH) for cross-build A/B (tools/ab_gemm_split.sh)."""
from __future__ import annotations

import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

SHAPES = [(4096, 4096, 4096, "KK", 256), (4096, 4096, 4096, "KN", 256), (4096, 4096, 4096, "MN", 256),
          (8192, 8192, 8192, "KK", 256), (3200, 32000, 2048, "KK", 0), (3200, 2048, 32000, "KN", 0),
          (32000, 2048, 3200, "MN", 0), (4096, 512, 2048, "KK", 0), (4096, 2048, 512, "KK", 0)]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
    T = _lib.ops()
    T.gemm_lib_policy(0)
    dev = torch.device("cuda", 0)
    for M, N, K, lay, sched in SHAPES:
        ak, bk = lay[0] == "K", lay[1] == "K"
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(K, N, device=dev) * 2 - 1).to(torch.bfloat16)
        a_ = A if ak else A.t().contiguous()
        b_ = B.t().contiguous() if bk else B
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        T.gemm8p_policy(2 if sched else 1, sched)
        fn = lambda: T.gemm(a_, ak, b_, bk, c, 0, None, False, None, 1.0, False)  # noqa: E731
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / 10)
        print(json.dumps({"lib": tag, "shape": f"{M}x{N}x{K} {lay}", "ms": round(best, 4),
                          "tflops": round(2.0 * M * N * K / best / 1e9, 1)}), flush=True)
    T.gemm8p_policy(1, 0)


if __name__ == "__main__":
    main()
