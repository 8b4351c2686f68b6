"""Why 4096^3 bf16 read 1169-1204 TF/s in round 2 and 1088-1095 in round 3:
the SAME kernel (gemm8p 256^2, schedule 4, K-major x K-major) timed under
both rounds' measurement protocols in one process, plus a sustained run and
zero-filled operands, next to hipBLASLt (torch.mm) under the same protocols.

  r2 protocol (tools/ab_gemm8p_sched.py, round 2): 2 warm calls, ONE timed
     burst of 10 calls per round, variants interleaved -> median of 6 rounds
  r3 protocol (tools/gemm_shapes_tf.py, round 3): 5 warm calls, best of 5
     back-to-back bursts of 10 calls
  sustained: 500 back-to-back calls after 50 warm ones (clock/power steady state)

    python tools/gemm_4096_protocols.py [--out profiles/r4/gemm4096_protocols.json]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

M = N = K = 4096
FL = 2.0 * M * N * K


def burst(fn, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return FL / (e0.elapsed_time(e1) / n / 1e3) / 1e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    T = _lib.ops()
    T.gemm_lib_policy(0)
    dev = torch.device("cuda", 0)
    data = {"uniform": lambda: (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16),
            "zeros": lambda: torch.zeros(M, K, device=dev, dtype=torch.bfloat16)}
    out = {}
    for dname, mk in data.items():
        A, B = mk(), mk()
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

        def ours():
            T.gemm(A, True, B, True, c, 0, None, False, None, 1.0, False)

        def lib():
            torch.mm(A, B.t(), out=c)

        T.gemm8p_policy(2, 256)          # forced 256^2 tile (the production schedule)
        fns = {"gemm8p": ours, "hipblaslt": lib}
        r2 = {k: [] for k in fns}
        for _ in range(6):               # r2: interleaved, 2 warm + one burst of 10
            for k, fn in fns.items():
                fn(); fn()
                r2[k].append(burst(fn, 10))
        r3 = {}
        for k, fn in fns.items():        # r3: 5 warm + best of 5 bursts of 10
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            r3[k] = max(burst(fn, 10) for _ in range(5))
        sus = {}
        for k, fn in fns.items():
            for _ in range(50):
                fn()
            torch.cuda.synchronize()
            sus[k] = burst(fn, 500)
        T.gemm8p_policy(1, 0)
        for k in fns:
            out[f"{dname}/{k}"] = {"r2_median": round(statistics.median(r2[k]), 1),
                                   "r2_best": round(max(r2[k]), 1), "r3_best": round(r3[k], 1),
                                   "sustained_500": round(sus[k], 1)}
            print(json.dumps({f"{dname}/{k}": out[f"{dname}/{k}"]}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
