"""Per-model training throughput on one MI355X through the tiresias_amd
kernels (samples/s and ms/step), with a rocprof-friendly fixed step count.
These per-iteration times are also what the cluster simulator's job model
uses (``--throughput_table``)."""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.executor.trainer import Trainer  # noqa: E402


def bench(model, batch=None, steps=10, warmup=3, graph=False, overlap=None, branches=None):
    dev = torch.device("cuda", 0)
    t = Trainer(model, dev, batch=batch, use_graph=graph, overlap_wgrad=overlap,
                branches=branches)
    for _ in range(warmup):
        t.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        t.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return dict(model=model, batch=t.batch, graph=graph, overlap_wgrad=t.overlap_wgrad, branches=t.branches, ms_per_step=dt * 1e3,
                samples_per_s=t.samples_per_step() / dt, loss=float(t.last_loss),
                params=t.arena.numel, state_mb=t.state_bytes() / 2 ** 20)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="resnet50,vgg16,transformer,gnmt")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch override (0: the model default)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--overlap", type=int, default=-1,
                    help="weight gradients on a side stream: -1 per-model default, 0 off, 1 on")
    ap.add_argument("--branches", type=int, default=-1,
                    help="model branch streams (GNMT's independent recurrences): -1 model default, 0 off, 1 on")
    ap.add_argument("--lib", type=int, default=None,
                    help="plain-GEMM routing: -1 measured MFMA/hipBLASLt (production default), 0 MFMA only, "
                         "1 library; unset: the library default")
    ap.add_argument("--conv_policy", type=int, default=1,
                    help="conv core: 1 LDS-DMA where the cost model picks it, 2 wherever eligible, 0 igemm only")
    ap.add_argument("--save_routes", default=None,
                    help="write the routing table (shipped decisions + the shapes tuned in this run) here")
    ap.add_argument("--policy", action="append", default=[],
                    help="name=value: call torch.ops.tam.<name>(value) before the runs (A/B switches, "
                         "e.g. conv_stem_policy=0); repeatable")
    ap.add_argument("--conv_split", type=int, default=1,
                    help="split-K of under-filled LDS-DMA conv passes: 1 on (default), 0 off")
    a = ap.parse_args()
    import torch
    from tiresias_amd.ops import _lib
    _lib.load(required=True)
    if a.lib is not None:
        torch.ops.tam.gemm_lib_policy(a.lib)
    torch.ops.tam.conv_dma_policy(a.conv_policy)
    torch.ops.tam.conv_split_policy(a.conv_split)
    for kv in a.policy:
        k, v = kv.split("=")
        getattr(torch.ops.tam, k)(int(v))
    res = []
    for m in a.models.split(","):
        r = bench(m, batch=a.batch or None, steps=a.steps, warmup=a.warmup, graph=a.graph,
                  overlap=None if a.overlap < 0 else bool(a.overlap), branches=None if a.branches < 0 else bool(a.branches))
        print(json.dumps(r), flush=True)
        res.append(r)
    routes = torch.ops.tam.gemm_routes().strip().splitlines()
    print(f"gemm routes ({sum('lib' in r for r in routes)} of {len(routes)} plain-GEMM shapes -> hipBLASLt):")
    print("\n".join(routes))
    if a.save_routes:
        print("routes ->", _lib.save_routes(a.save_routes), flush=True)
    if a.out:
        json.dump({"models": res, "lib_policy": a.lib, "conv_split": a.conv_split, "gemm_routes": routes}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
