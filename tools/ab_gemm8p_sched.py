"""A/B of gemm8p schedule variants in ONE process, interleaved rounds
(guide §5.4 rule 24): 256^2 tile, random operands. Prints median / best
TFLOP/s per variant and shape."""
import json
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

T = _lib.ops()
T.gemm_lib_policy(0)
dev = torch.device("cuda", 0)
# variant "s" = schedule s (group 4); "s:g" = schedule s with tile-order group g
variants = [v for v in (sys.argv[1] if len(sys.argv) > 1 else "0,2,3").split(",")]
res = {}
for (M, N, K) in [(4096, 4096, 4096), (8192, 8192, 8192)]:
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ref = None
    times = {v: [] for v in variants}
    for rnd in range(6):
        for v in variants:
            sch, grp = (int(x) for x in (v.split(":") + ["4"])[:2])
            T.gemm8p_policy(2, 200 + sch)        # forced 256^2 tile, schedule sch, no split
            T.gemm8p_group(grp)
            for _ in range(2):
                T.gemm(A, True, B, True, c, 0, None, False, None, 1.0, False)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                T.gemm(A, True, B, True, c, 0, None, False, None, 1.0, False)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(2.0 * M * N * K / (e0.elapsed_time(e1) / 10 / 1e3) / 1e12)
            if ref is None:
                ref = c.float().clone()
            else:
                err = ((c.float() - ref).norm() / ref.norm()).item()
                assert err < 1e-3, (v, err)
    res[f"{M}x{N}x{K}"] = {v: {"median_tf": round(statistics.median(t), 1), "best_tf": round(max(t), 1)}
                           for v, t in times.items()}
T.gemm8p_policy(1, 4)
T.gemm8p_group(4)
print(json.dumps(res))
