"""GNMT step time with 1 vs N arrival counters per batch tile in the
persistent LSTM recurrence (tam.lstm_seq_shards): one hipGraph-captured
trainer per setting (the shard count is baked into each capture), timed in
interleaved rounds in one process."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.executor.trainer import Trainer  # noqa: E402
from tiresias_amd.ops import _lib  # noqa: E402

_lib.load(required=True)
dev = torch.device("cuda", 0)
settings = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,4").split(",")]
tr = {}
for ns in settings:
    torch.ops.tam.lstm_seq_shards(ns)
    t = Trainer("gnmt", dev, seed=3, use_graph=True)
    for _ in range(4):                 # 2 eager warm steps + capture + 1 replay
        t.step()
    tr[ns] = t
torch.cuda.synchronize()
res = {ns: [] for ns in settings}
for _ in range(5):
    for ns in settings:
        t = tr[ns]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            t.step()
        torch.cuda.synchronize()
        res[ns].append((time.perf_counter() - t0) / 10 * 1e3)
from tiresias_amd.models import gnmt as G  # noqa: E402

print(json.dumps({"ms_per_step": {str(k): sorted(v) for k, v in res.items()},
                  "median": {str(k): sorted(v)[len(v) // 2] for k, v in res.items()},
                  "persist_errors": G.persist_errors()}))
