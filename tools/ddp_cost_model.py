"""N-GPU step-time ESTIMATES (a cost model, not a measurement) for the data-
parallel wire formats of parallel/ddp.py: fp32 all-reduce (default), sharded
fp32 (reduce-scatter fp32 + bf16 shadow all-gather, 1/N optimizer) and
sharded bf16 (reduce-scatter bf16 + all-gather bf16).

Inputs are the MEASURED one-GPU numbers (hipGraph step = forward + backward
+ optimizer, and the optimizer kernel's share of it, from the rocprofv3
profiles) plus an ASSUMED RCCL ring bus bandwidth over xGMI (MI355X: 7
point-to-point links of ~153 GB/s per GPU; the achievable ring bus
bandwidth is not measured on this 1-GPU box -- the table brackets it).
A ring collective over N ranks moves, per member,
  all-reduce      2 (N-1)/N x S
  reduce-scatter  (N-1)/N   x S,   all-gather (N-1)/N x S
so t = bytes_per_member / busbw. Overlap: the gradient reduction overlaps
backward except the LAST bucket (bucket_mb); the all-gather of the sharded
modes runs after the optimizer, not overlapped.

    python tools/ddp_cost_model.py [--n 8] [--busbw 150,300,450] [--out profiles/r4/ddp_cost_model.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# one-GPU hipGraph steps (ms) and optimizer share measured on MI355X
# (profiles/r3/s3/*_graph_kernel_stats_*.csv, profiles/r4/*), parameters
MODELS = {
    "vgg16": dict(step_ms=7.52, opt_frac=0.079, params=138.4e6, bwd_frac=0.62),
    "gnmt": dict(step_ms=10.60, opt_frac=0.145, params=226.6e6, bwd_frac=0.55),
    "resnet50": dict(step_ms=9.88, opt_frac=0.010, params=25.6e6, bwd_frac=0.62),
    "transformer": dict(step_ms=5.42, opt_frac=0.071, params=60.5e6, bwd_frac=0.55),
}


def estimate(m: dict, n: int, busbw_gbs: float, mode: str, bucket_mb: float = 32.0) -> dict:
    P = m["params"]
    opt_ms = m["step_ms"] * m["opt_frac"]
    compute_ms = m["step_ms"] - opt_ms
    bwd_ms = compute_ms * m["bwd_frac"]
    f = (n - 1) / n
    bw = busbw_gbs * 1e9
    if mode == "allreduce":
        grad_b, gather_b, opt = 2 * f * 4 * P, 0.0, opt_ms
        last = 2 * f * min(bucket_mb * 2 ** 20, 4 * P)
    elif mode == "shard_fp32":
        grad_b, gather_b, opt = f * 4 * P, f * 2 * P, opt_ms / n
        last = f * min(bucket_mb * 2 ** 20, 4 * P)
    elif mode == "shard_bf16":
        grad_b, gather_b, opt = f * 2 * P, f * 2 * P, opt_ms / n
        last = f * min(bucket_mb * 2 ** 20, 4 * P) / 2
    else:
        raise ValueError(mode)
    grad_ms = grad_b / bw * 1e3
    # reduction hidden behind backward except what exceeds it + the last bucket
    exposed = max(grad_ms - bwd_ms, 0.0) + last / bw * 1e3
    gather_ms = gather_b / bw * 1e3
    step = compute_ms + exposed + opt + gather_ms
    return dict(mode=mode, wire_mb_per_member=round((grad_b + gather_b) / 2 ** 20, 1),
                grad_comm_ms=round(grad_ms, 3), exposed_ms=round(exposed, 3), optimizer_ms=round(opt, 3),
                gather_ms=round(gather_ms, 3), step_ms=round(step, 3),
                vs_1gpu=round(step / m["step_ms"], 3))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--busbw", default="150,300,450", help="assumed RCCL ring bus bandwidth, GB/s")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r4", "ddp_cost_model.json"))
    a = ap.parse_args()
    rows = []
    for name, m in MODELS.items():
        for bb in (float(x) for x in a.busbw.split(",")):
            for mode in ("allreduce", "shard_fp32", "shard_bf16"):
                r = estimate(m, a.n, bb, mode)
                r.update(model=name, n=a.n, busbw_gbs=bb)
                rows.append(r)
    out = {"what": "COST-MODEL estimates (not measurements) of the N-GPU DDP step per wire format; "
                   "1-GPU inputs measured on MI355X, bus bandwidth assumed (bracketed)",
           "models": MODELS, "rows": rows}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print("| model | busbw GB/s | mode | wire MB/member | exposed ms | optimizer ms | gather ms | step ms |")
    print("|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['model']} | {r['busbw_gbs']:.0f} | {r['mode']} | {r['wire_mb_per_member']} | {r['exposed_ms']} | "
              f"{r['optimizer_ms']} | {r['gather_ms']} | {r['step_ms']} |")


if __name__ == "__main__":
    main()
