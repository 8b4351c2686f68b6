"""Diagnostic: per-step losses of a full-size model in eager and/or hipGraph
replay mode, each in a FRESH trainer (finds graph-only numerics faults).

    python tools/diag_graph.py --model resnet50 --steps 14 --modes graph,eager
"""
import argparse
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.executor.trainer import Trainer  # noqa: E402
from tiresias_amd.ops import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="resnet50")
ap.add_argument("--steps", type=int, default=8)
ap.add_argument("--seed", type=int, default=0)
ap.add_argument("--modes", default="graph,eager")
ap.add_argument("--policy", type=int, default=1)
ap.add_argument("--nosync", action="store_true", help="no host sync between steps")
a = ap.parse_args()
_lib.load(required=True)
_lib.ops().conv_dma_policy(a.policy)
for mode in a.modes.split(","):
    t = Trainer(a.model, "cuda", seed=a.seed, use_graph=(mode == "graph"))
    if a.nosync:
        ls = [t.step().detach().clone() for _ in range(a.steps)]
        ls = [round(float(x), 3) for x in ls]
    else:
        ls = [round(float(t.step()), 3) for _ in range(a.steps)]
    ls.append(("last", round(float(t.last_loss), 3)))
    print(f"{mode}: losses={ls} |w|={float(t.arena.master.norm()):.3f}", flush=True)
    del t
    torch.cuda.empty_cache()
