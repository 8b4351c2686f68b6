"""Every GEMM shape the four models actually run (the shipped routing table,
profiles/gemm_routes_<device>.txt) through our routed kernels vs hipBLASLt
(ATen mm on the same memory layouts, fp32 output where the model's GEMM
accumulates into fp32 grads). Random uniform bf16 operands (guide §5.4 rule
25). Prints one JSON line per shape and a time-weighted summary: where the
remaining gap to the library is, weighted by how long the models spend there.

    python tools/bench_gemm_routes.py [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

BF = torch.bfloat16


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--min-mflop", type=float, default=100.0, help="skip tiny GEMMs")
    ap.add_argument("--save", default=None, help="write this process's routing decisions here (run with "
                    "TAM_GEMM_ROUTES=0 to re-tune every shape instead of loading the shipped table)")
    a = ap.parse_args()
    T = _lib.ops()
    dev = torch.device("cuda", 0)
    rows = []
    keys = []
    for ln in _lib.routes_file().read_text().splitlines():
        p = ln.split()
        if len(p) < 8:
            continue
        M, N, K = int(p[0]), int(p[1]), int(p[2])
        keys.append((M, N, K, p[3][0] == "K", p[3][1] == "K", int(p[4]), p[5] == "1", p[7]))
    for M, N, K, ak, bk, mode, f32, route in keys:
        fl = 2.0 * M * N * K
        if fl / 1e6 < a.min_mflop:
            continue
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(BF)
        B = (torch.rand(K, N, device=dev) * 2 - 1).to(BF)
        a_ = A if ak else A.t().contiguous()          # K-major [M][K] or M-major [K][M]
        b_ = B.t().contiguous() if bk else B          # K-major [N][K] or N-major [K][N]
        c = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else BF)
        ours = timeit(lambda: T.gemm(a_, ak, b_, bk, c, mode, None, False, None, 1.0, True))
        Ae = a_ if ak else a_.t()
        Be = b_.t() if bk else b_
        if f32:
            lib = timeit(lambda: torch.mm(Ae, Be, out_dtype=torch.float32))
        else:
            lib = timeit(lambda: torch.mm(Ae, Be))
        r = {"shape": f"{M}x{N}x{K} {'K' if ak else 'M'}{'K' if bk else 'N'}", "mode": mode, "f32": f32,
             "route": route, "ours_us": round(ours * 1e3, 2), "lib_us": round(lib * 1e3, 2),
             "ours_tflops": round(fl / ours / 1e9, 1), "lib_tflops": round(fl / lib / 1e9, 1),
             "ratio": round(lib / ours, 3)}
        print(json.dumps(r), flush=True)
        rows.append(r)
    tot_o = sum(r["ours_us"] for r in rows)
    tot_l = sum(r["lib_us"] for r in rows)
    print(json.dumps({"summary": "sum over shapes (one call each)", "ours_us": round(tot_o, 1),
                      "lib_us": round(tot_l, 1), "ratio": round(tot_l / tot_o, 3)}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    if a.save:
        with open(a.save, "w") as f:
            f.write(T.gemm_routes())


if __name__ == "__main__":
    main()
