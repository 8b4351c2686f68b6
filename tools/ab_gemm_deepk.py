"""Deep-K, few-tile GEMMs (vocab-projection input gradients, KN layout, bf16
out): gemm8p tile x slab-split x tile-order group, interleaved rounds in one
process. Prints median TFLOP/s per variant and shape."""
import json
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

T = _lib.ops()
T.gemm_lib_policy(0)
dev = torch.device("cuda", 0)
variants = [(256, 1, 4), (256, 2, 4), (256, 3, 4), (256, 4, 4), (256, 5, 4), (256, 8, 4),
            (256, 2, 1), (256, 2, 13), (256, 5, 1), (256, 5, 13), (128, 1, 4), (128, 2, 4), (128, 3, 4)]
res = {}
for (M, N, K) in [(3200, 2048, 32000), (3200, 2048, 4096), (3200, 1024, 4096)]:
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)        # K-major [M][K]
    B = (torch.rand(K, N, device=dev) * 2 - 1).to(torch.bfloat16)        # N-major [K][N]
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ref = (A.float() @ B.float())
    times = {v: [] for v in variants}
    for rnd in range(4):
        for v in variants:
            tile, sp, grp = v
            T.gemm8p_policy(3, (200 if tile == 256 else 100) + 4)
            T.gemm8p_slab_force(sp)
            T.gemm8p_group(grp)
            for _ in range(2):
                T.gemm(A, True, B, False, c, 0, None, False, None, 1.0, False)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                T.gemm(A, True, B, False, c, 0, None, False, None, 1.0, False)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(2.0 * M * N * K / (e0.elapsed_time(e1) / 10 / 1e3) / 1e12)
            if rnd == 0:
                err = ((c.float() - ref).norm() / ref.norm()).item()
                assert err < 1e-2, (v, err)
    res[f"{M}x{N}x{K} KN"] = {f"t{v[0]}_sp{v[1]}_g{v[2]}": round(statistics.median(t), 1) for v, t in times.items()}
T.gemm8p_policy(1, 4)
T.gemm8p_slab_force(0)
T.gemm8p_group(4)
print(json.dumps(res, indent=1))
