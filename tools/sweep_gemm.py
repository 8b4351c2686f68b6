"""Sweep the MFMA GEMM's tile config x split-K over the GEMM shapes the model
zoo actually issues (fwd / dgrad / wgrad of every linear layer), against the
heuristic and hipBLASLt (torch.matmul). Output: one JSON line per shape with
the best (cfg, splits), used to set ``choose_tiles`` in csrc/include/tam/tiles.h.
"""
from __future__ import annotations

import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

BF = torch.bfloat16
CFG = {0: "128x128", 1: "128x64", 2: "64x128", 3: "64x64", 4: "256x256"}


def model_shapes():
    """(name, M, N, K, a_kmajor, b_kmajor, fp32_out) for the zoo's linears."""
    out = []
    lin = {  # name: (tokens, in, out)
        "tf.qkv": (4096, 512, 1536), "tf.proj": (4096, 512, 512), "tf.ffn1": (4096, 512, 2048),
        "tf.ffn2": (4096, 2048, 512), "tf.logits": (4096, 512, 32000),
        "gn.xproj": (3200, 1024, 4096), "gn.xproj2": (3200, 2048, 4096), "gn.attn": (3200, 1024, 1024),
        "gn.logits": (3200, 1024, 32000), "vgg.fc1": (32, 25088, 4096), "rn.fc": (64, 2048, 1000),
        "gn.rec": (64, 1024, 4096),
    }
    for n, (T, I, O) in lin.items():
        out.append((n + ".fwd", T, O, I, True, True, n == "gn.xproj" or n == "gn.rec"))
        out.append((n + ".dgrad", T, I, O, True, False, n == "gn.rec"))
        out.append((n + ".wgrad", O, I, T, False, False, True))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    _lib.load(required=True)
    T = torch.ops.tam
    T.gemm_lib_policy(0)   # measure the MFMA kernels themselves
    dev = torch.device("cuda", 0)
    res = []
    for (name, M, N, K, ak, bk, f32) in model_shapes():
        if a.only and a.only not in name:
            continue
        A = torch.randn(M, K, device=dev).to(BF)
        B = torch.randn(K, N, device=dev).to(BF)
        aa = A if ak else A.t().contiguous()
        bb = B.t().contiguous() if bk else B
        c = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else BF)
        mode = 1 if f32 else 0

        def run():
            T.gemm(aa, ak, bb, bk, c, mode, None, False, None, 1.0, f32)

        fl = 2.0 * M * N * K
        T.gemm_force(-1, -1)
        t_auto = timeit(run, iters=10, warmup=3)
        best = (t_auto, "auto")
        grid = {}
        for cfg in range(5):
            if cfg == 4 and not (ak and bk and K % 64 == 0 and M >= 128 and N >= 128):
                continue
            for sp in ((1, 2, 4, 8, 16, 32) if f32 else (1,)):
                T.gemm_force(cfg, sp)
                t = timeit(run, iters=10, warmup=2)
                grid[f"{CFG[cfg]}/s{sp}"] = round(fl / t / 1e9, 1)
                if t < best[0]:
                    best = (t, f"{CFG[cfg]}/s{sp}")
        T.gemm_force(-1, -1)
        at = aa if ak else aa.t()
        bt = bb.t() if bk else bb
        t_ref = timeit(lambda: torch.matmul(at, bt), iters=10, warmup=3)
        r = dict(name=name, M=M, N=N, K=K, layout=("K" if ak else "M") + ("K" if bk else "N"),
                 f32=f32, auto_tflops=round(fl / t_auto / 1e9, 1), best=best[1],
                 best_tflops=round(fl / best[0] / 1e9, 1), hipblaslt_tflops=round(fl / t_ref / 1e9, 1),
                 grid=grid)
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
