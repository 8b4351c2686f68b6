"""Per-parameter gradient comparison of a model's GPU kernels vs the fp32
CPU reference path (same weights, same batch)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.executor.trainer import Trainer  # noqa: E402


def main(model="resnet_tiny", **kw):
    dev = torch.device("cuda", 0)
    tg = Trainer(model, dev, seed=3, model_kwargs=kw or None)
    tc = Trainer(model, "cpu", seed=3, model_kwargs=kw or None)
    tc.arena.master.copy_(tg.arena.master.cpu())
    tc.arena.shadow.copy_(tg.arena.shadow.cpu())
    tc.data = {k: v.cpu() for k, v in tg.data.items()}
    lg, lc = float(tg._fwd_bwd()), float(tc._fwd_bwd())
    print(f"{model} {kw} loss gpu={lg:.5f} cpu={lc:.5f}")
    gg = tg.arena.grad.cpu()
    tot = ((gg - tc.arena.grad).norm() / tc.arena.grad.norm()).item()
    print(f"total rel err {tot:.4f}")
    rows = []
    for p in tg.arena.params:
        a = gg[p.offset:p.offset + p.numel]
        b = tc.arena.grad[p.offset:p.offset + p.numel]
        rows.append(((a - b).norm().item(), (a - b).norm().item() / (b.norm().item() + 1e-12), b.norm().item(), p.name))
    for r in sorted(rows, reverse=True)[:12]:
        print(f"  abs {r[0]:.3e} rel {r[1]:.3e} |ref| {r[2]:.3e} {r[3]}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "resnet_tiny")
