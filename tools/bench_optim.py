"""Fused optimizer kernels (csrc/kernels/optim.hip) on the model arenas'
sizes: achieved HBM bandwidth of one SGD-momentum / AdamW step (bytes =
master+grad+state reads, master+state+grad-zero+bf16 shadow writes)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tiresias_amd.ops import _lib  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3        # us


def main():
    _lib.load(required=True)
    T = _lib.ops()
    dev = torch.device("cuda", 0)
    out = []
    variants = [int(v) for v in os.environ.get("OPTIM_VARIANTS", "0,3").split(",")]
    grids = [int(v) for v in os.environ.get("OPTIM_GRIDS", "0").split(",")]
    for name, n, opt in [("vgg16", 138360448, "sgd"), ("resnet50", 25572736, "sgd"),
                         ("gnmt", 226561280, "adam"), ("transformer", 60524544, "adam")]:
        w = torch.randn(n, device=dev); g = torch.randn(n, device=dev)
        m = torch.zeros(n, device=dev); wb = torch.empty(n, device=dev, dtype=torch.bfloat16)
        v = torch.zeros(n, device=dev) if opt == "adam" else None
        for var, grid in [(v_, g_) for v_ in variants for g_ in grids] * 2:   # two interleaved rounds
            T.optim_variant(var)
            T.optim_grid(grid)
            if opt == "sgd":
                us = timeit(lambda: T.sgd_step(w, g, m, wb, 0.1, 0.9, 1e-4, 1.0, False, True))
                nbytes = n * (12 + 12 + 2)
            else:
                us = timeit(lambda: T.adam_step(w, g, m, v, wb, 1e-3, 0.9, 0.98, 1e-9, 0.01, 3, 1.0, True))
                nbytes = n * (16 + 16 + 2)
            r = dict(model=name, opt=opt, variant=var, grid=grid, params=n, us=round(us, 1),
                     tb_per_s=round(nbytes / us / 1e6, 2))
            print(json.dumps(r), flush=True)
            out.append(r)
        T.optim_variant(-1)
        T.optim_grid(0)
        del v
        del w, g, m, wb
        torch.cuda.empty_cache()
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
