"""4-wave 256^2 GEMM (gemm4w) vs gemm8p (8-wave, schedule 4) on K-major x
K-major bf16, interleaved rounds in one process; checks numerics first."""
import json
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

T = _lib.ops()
T.gemm_lib_policy(0)
dev = torch.device("cuda", 0)
res = {}
shapes = [(4096, 4096, 4096), (8192, 8192, 8192), (3200, 4096, 1024), (4096, 2048, 3200), (3000, 1000, 640)]
for (M, N, K) in shapes:
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ref = A.float() @ B.float().t()
    assert T.gemm4w(A, B, c, 1)
    torch.cuda.synchronize()
    err = ((c.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, (M, N, K, err)
    if M % 256 or N % 256:
        res[f"{M}x{N}x{K}"] = {"rel_err": err}
        continue
    times = {"gemm4w_p0": [], "gemm4w_p1": [], "gemm8p": []}
    for rnd in range(6):
        for v in times:
            if v == "gemm8p":
                T.gemm8p_policy(2, 204)
                fn = lambda: T.gemm(A, True, B, True, c, 0, None, False, None, 1.0, False)
            else:
                pipe = int(v[-1])
                fn = lambda: T.gemm4w(A, B, c, pipe)
            for _ in range(2):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[v].append(2.0 * M * N * K / (e0.elapsed_time(e1) / 10 / 1e3) / 1e12)
    res[f"{M}x{N}x{K}"] = {v: {"median_tf": round(statistics.median(t), 1), "best_tf": round(max(t), 1)}
                           for v, t in times.items()}
    res[f"{M}x{N}x{K}"]["rel_err"] = err
T.gemm8p_policy(1, 4)
print(json.dumps(res, indent=1))
