"""VGG-16 step A/B of the patch-staged wgrad (tam.conv_wgrad_c64_policy 1 vs
0) in one process, for the hipGraph 1-GPU trainer (weight gradients on the
side stream: the patch kernel is kept off it) and the eager gang-path
trainer (no side stream); trainers built once per policy, steps interleaved."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.executor.trainer import Trainer  # noqa: E402
from tiresias_amd.ops import _lib  # noqa: E402

T = _lib.ops()
dev = torch.device("cuda", 0)
out = {}
for mode, kw in (("graph", dict(use_graph=True)), ("eager_no_side_stream", dict(use_graph=False, overlap_wgrad=False))):
    trainers = {}
    for pol in (1, 0):
        T.conv_wgrad_c64_policy(pol)
        t = Trainer("vgg16", dev, seed=0, **kw)
        for _ in range(4):
            t.step()
        torch.cuda.synchronize()
        trainers[pol] = t
    res = {}
    for rnd in range(3):
        for pol, t in trainers.items():
            T.conv_wgrad_c64_policy(pol)          # (eager: read at each launch)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                t.step()
            torch.cuda.synchronize()
            res.setdefault(pol, []).append(round((time.perf_counter() - t0) / 20 * 1e3, 3))
    out[mode] = {"c64_on_ms": res[1], "c64_off_ms": res[0]}
    del trainers
    torch.cuda.empty_cache()
T.conv_wgrad_c64_policy(1)
print(json.dumps(out))
