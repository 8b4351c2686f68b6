"""Kernel micro-benchmarks: tiresias_amd HIP kernels vs the vendor libraries
PyTorch-ROCm dispatches to (hipBLASLt GEMM, MIOpen conv, SDPA attention).
Same random bf16 data for both (guide §5.4 rule 25). Prints one JSON line per
case and a summary table; ``--out`` writes the JSON list.
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

BF = torch.bfloat16


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(3):
        ev[0].record()
        for _ in range(iters):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) / iters)
    return min(ts)


BIG_GEMMS = [(4096, 4096, 4096, True, True), (8192, 8192, 8192, True, True),
             (4096, 4096, 4096, True, False), (4096, 4096, 4096, False, False),
             (16384, 2048, 512, True, True), (4096, 32000, 512, True, True),
             (512, 2048, 16384, False, False)]
# the zoo's small/medium linears: Transformer-base (4096 tokens) fwd KK / dgrad
# KN / wgrad MN, GNMT LSTM recurrence (batch 64) and its projections
ZOO_GEMMS = [(4096, 512, 512, True, True), (4096, 1536, 512, True, True),
             (4096, 2048, 512, True, True), (4096, 512, 2048, True, True),
             (4096, 512, 512, True, False), (4096, 512, 2048, True, False),
             (4096, 2048, 512, True, False), (512, 512, 4096, False, False),
             (2048, 512, 4096, False, False), (512, 2048, 4096, False, False),
             (64, 4096, 1024, True, True), (64, 1024, 4096, True, False),
             (3200, 4096, 1024, True, True), (1024, 4096, 3200, False, False)]


def gemm_cases(T, dev, shapes=BIG_GEMMS):
    out = []
    for (M, N, K, ak, bk) in shapes:
        A = torch.randn(M, K, device=dev).to(BF)
        B = torch.randn(K, N, device=dev).to(BF)
        a = A if ak else A.t().contiguous()
        b = B.t().contiguous() if bk else B
        c = torch.empty(M, N, device=dev, dtype=BF)
        t_ours = timeit(lambda: T.gemm(a, ak, b, bk, c, 0, None, False, None, 1.0, False))
        at = a if ak else a.t()
        bt = b.t() if bk else b
        t_ref = timeit(lambda: torch.matmul(at, bt))
        fl = 2.0 * M * N * K
        out.append(dict(kind="gemm", shape=f"{M}x{N}x{K} {'K' if ak else 'M'}{'K' if bk else 'N'}",
                        ours_ms=t_ours, ref_ms=t_ref, ours_tflops=fl / t_ours / 1e9,
                        ref_tflops=fl / t_ref / 1e9))
    return out


RESNET_CONVS = [  # N,H,C,K,R,stride,pad   (batch 64)
    (64, 56, 64, 64, 3, 1, 1), (64, 56, 64, 256, 1, 1, 0), (64, 56, 256, 64, 1, 1, 0),
    (64, 56, 128, 128, 3, 2, 1), (64, 28, 128, 128, 3, 1, 1), (64, 28, 512, 128, 1, 1, 0),
    (64, 14, 256, 256, 3, 1, 1), (64, 14, 1024, 256, 1, 1, 0), (64, 7, 512, 512, 3, 1, 1),
    (64, 224, 8, 64, 7, 2, 3), (64, 56, 256, 512, 1, 2, 0),
]


VGG_CONVS = [  # batch 32, every distinct VGG-16 conv (first layer: RGB padded to 8 channels)
    (32, 224, 8, 64, 3, 1, 1), (32, 224, 64, 64, 3, 1, 1), (32, 112, 64, 128, 3, 1, 1),
    (32, 112, 128, 128, 3, 1, 1), (32, 56, 128, 256, 3, 1, 1), (32, 56, 256, 256, 3, 1, 1),
    (32, 28, 256, 512, 3, 1, 1), (32, 28, 512, 512, 3, 1, 1), (32, 14, 512, 512, 3, 1, 1),
]


def conv_cases(T, dev, shapes=RESNET_CONVS):
    out = []
    for (N, H, C, K, R, st, pd) in shapes:
        x = torch.randn(N, H, H, C, device=dev).to(BF)
        w = (torch.randn(K, R, R, C, device=dev) * 0.05).to(BF)
        P = (H + 2 * pd - R) // st + 1
        y = torch.empty(N, P, P, K, device=dev, dtype=BF)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        wt = torch.empty_like(w)
        dw = torch.zeros(K, R, R, C, device=dev)
        t_f = timeit(lambda: T.conv_fwd(x, w, y, st, pd, 1, None, False))
        t_d = timeit(lambda: T.conv_dgrad(dy, w, wt, dx, st, pd, 1, None))
        t_w = timeit(lambda: T.conv_wgrad(dy, x, dw, st, pd, 1, 0))
        # vendor: channels_last NCHW view through MIOpen
        xr = x.permute(0, 3, 1, 2)
        wr = w.permute(0, 3, 1, 2)
        dyr = dy.permute(0, 3, 1, 2)
        rf = timeit(lambda: F.conv2d(xr, wr, stride=st, padding=pd))
        xg = xr.detach().requires_grad_(True)
        wg = wr.detach().requires_grad_(True)
        yv = F.conv2d(xg, wg, stride=st, padding=pd)
        rb = timeit(lambda: torch.autograd.grad(yv, [xg, wg], dyr, retain_graph=True))
        fl = 2.0 * N * P * P * K * R * R * C
        out.append(dict(kind="conv", shape=f"N{N} H{H} C{C} K{K} R{R} s{st}",
                        fwd_ms=t_f, dgrad_ms=t_d, wgrad_ms=t_w, ref_fwd_ms=rf, ref_bwd_ms=rb,
                        fwd_tflops=fl / t_f / 1e9, dgrad_tflops=fl / t_d / 1e9,
                        wgrad_tflops=fl / t_w / 1e9, ref_fwd_tflops=fl / rf / 1e9,
                        ours_total_ms=t_f + t_d + t_w, ref_total_ms=rf + rb))
    return out


def attn_cases(T, dev):
    out = []
    for (B, H, S, causal) in [(32, 8, 128, False), (32, 8, 128, True), (16, 8, 512, False), (64, 16, 256, True)]:
        qkv = torch.randn(B, S, 3, H, 64, device=dev).to(BF)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        o = torch.empty(B, S, H, 64, device=dev, dtype=BF)
        lse = torch.empty(B, H, S, device=dev)
        t_f = timeit(lambda: T.attn_forward(q, k, v, o, lse, causal, 0.125, None))
        do = torch.randn_like(o)
        dqkv = torch.empty_like(qkv)
        acc = torch.empty(B, S, H, 64, device=dev)
        de = torch.empty(B, H, S, device=dev)
        t_b = timeit(lambda: T.attn_backward(q, k, v, o, do, lse, dqkv[:, :, 0], dqkv[:, :, 1],
                                             dqkv[:, :, 2], acc, de, causal, 0.125, None))
        qt, kt, vt = (t.permute(0, 2, 1, 3) for t in (q, k, v))
        rf = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal))
        fl = 4.0 * B * H * S * S * 64 * (0.5 if causal else 1.0)
        out.append(dict(kind="attn", shape=f"B{B} H{H} S{S} causal={causal}", fwd_ms=t_f,
                        bwd_ms=t_b, ref_fwd_ms=rf, fwd_tflops=fl / t_f / 1e9,
                        bwd_tflops=2.5 * fl / t_b / 1e9, ref_fwd_tflops=fl / rf / 1e9))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default="gemm,conv,attn")
    ap.add_argument("--conv-dma", type=int, default=1, help="conv_dma_policy (0: igemm only)")
    ap.add_argument("--gemm-dma", type=int, default=0,
                    help="gemm_dma_policy: 0 igemm/gemm256, 2 LDS-DMA GEMM forced, 1 measured routing")
    a = ap.parse_args()
    _lib.load(required=True)
    T = torch.ops.tam
    T.gemm_lib_policy(0)   # measure the MFMA kernels themselves
    T.conv_dma_policy(a.conv_dma)
    T.gemm_dma_policy(a.gemm_dma, -1)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    res = []
    for kind in a.only.split(","):
        fn = {"gemm": gemm_cases, "conv": conv_cases, "attn": attn_cases,
              "vggconv": lambda T, d: conv_cases(T, d, VGG_CONVS),
              "zoogemm": lambda T, d: gemm_cases(T, d, ZOO_GEMMS)}[kind]
        for r in fn(T, dev):
            print(json.dumps(r), flush=True)
            res.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
