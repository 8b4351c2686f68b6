"""Isolate the MFMA GEMM's fixed per-tile cost (prologue + epilogue): time
fixed M x N at growing K for each tile config and output dtype."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

_lib.load(required=True)
T = torch.ops.tam
T.gemm_lib_policy(0)
dev = torch.device("cuda", 0)
BF = torch.bfloat16
M, N = 4096, 2048
for f32 in (False, True):
    for K in (64, 128, 256, 512, 1024, 2048):
        A = torch.randn(M, K, device=dev).to(BF)
        B = torch.randn(N, K, device=dev).to(BF)
        C = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else BF)
        row = {"f32": f32, "K": K}
        for cfg, name in ((3, "64x64"), (0, "128x128")):
            T.gemm_force(cfg, 1)
            row[name + "_us"] = round(timeit(lambda: T.gemm(A, True, B, True, C, 0, None, False, None, 1.0, False),
                                             iters=20, warmup=3) * 1e3, 2)
        T.gemm_force(-1, -1)
        print(json.dumps(row), flush=True)
