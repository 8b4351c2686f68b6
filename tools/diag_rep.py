"""Diagnostic: final loss of a 13-step full-size run under different host
synchronisation patterns, graph vs eager (isolates graph-replay races)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.executor.trainer import Trainer  # noqa: E402
from tiresias_amd.ops import _lib  # noqa: E402

_lib.load(required=True)
model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
variants = sys.argv[2].split(",") if len(sys.argv) > 2 else ["graph:devsync:1"]
for v in variants:
    mode, sync, pol = v.split(":")
    _lib.ops().conv_dma_policy(int(pol))
    t = Trainer(model, torch.device("cuda", 0), use_graph=(mode == "graph"))
    out = []
    for i in range(13):
        l = t.step()
        if sync == "devsync":
            torch.cuda.synchronize()
        elif sync == "streamsync":
            torch.cuda.current_stream().synchronize()
        elif sync == "item":
            out.append(round(float(l), 3))
    torch.cuda.synchronize()
    print(v, round(float(t.last_loss), 4), out[-4:], flush=True)
    del t
    torch.cuda.empty_cache()
