"""VGG-16 graph-step A/B of the patch-staged wgrad (tam.conv_wgrad_c64_policy
1 vs 0) in one process: both trainers captured once, replays interleaved."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.executor.trainer import Trainer  # noqa: E402
from tiresias_amd.ops import _lib  # noqa: E402

T = _lib.ops()
dev = torch.device("cuda", 0)
res = {}
trainers = {}
for pol in (1, 0):
    T.conv_wgrad_c64_policy(pol)
    t = Trainer("vgg16", dev, seed=0, use_graph=True)     # captured under this policy
    for _ in range(4):
        t.step()
    torch.cuda.synchronize()
    trainers[pol] = t
T.conv_wgrad_c64_policy(1)
for rnd in range(3):
    for pol, t in trainers.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            t.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 20 * 1e3
        res.setdefault(pol, []).append(round(ms, 3))
print(json.dumps({"c64_on_ms": res[1], "c64_off_ms": res[0]}))
