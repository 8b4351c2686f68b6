"""Per-job startup cost on one MI355X: Trainer construction, the eager warm
steps, hipGraph capture and steady-state steps, per model (each job pays the
startup once, so it adds directly to short jobs' JCT)."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.executor.trainer import Trainer  # noqa: E402
from tiresias_amd.ops import _lib  # noqa: E402


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return r, (time.perf_counter() - t0) * 1e3


def main():
    # TAM_GEMM_ROUTES=0: cold process WITHOUT the shipped routing table;
    # --save-routes: write this process's measured routes to the device table
    _lib.load(required=True)
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    models = args[0].split(",") if args else ["resnet50", "vgg16", "transformer", "gnmt"]
    out = []
    for rep in range(2):                     # rep 0 = cold process (route tuning etc.), rep 1 = warm
        for m in models:
            t, ms_init = timed(lambda: Trainer(m, torch.device("cuda", 0), seed=rep, use_graph=True))
            steps = [timed(t.step)[1] for _ in range(6)]
            r = dict(rep=rep, model=m, init_ms=round(ms_init, 2), step_ms=[round(s, 2) for s in steps])
            print(json.dumps(r), flush=True)
            out.append(r)
            _, ms_rel = timed(t.release)
            del t
    return out


if __name__ == "__main__":
    main()
    if "--save-routes" in sys.argv:
        print("routes ->", _lib.save_routes(), flush=True)
