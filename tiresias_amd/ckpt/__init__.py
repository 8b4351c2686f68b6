"""Checkpoint engine front-end.

``engine(dev)`` returns the native ``tam.CkptEngine`` (csrc/ckpt/ckpt_engine.cpp:
pinned host pool + low-priority side-stream hipMemcpyAsync spill / restore).
``measure(dev)`` times spill (D2H) and restore (H2D) through that engine over a
size sweep and writes the table the simulator's ``ckpt_policy=measured`` cost
model reads (``d2h_gbps`` / ``h2d_gbps`` / ``p2p_gbps``).

    python -m tiresias_amd.ckpt --out profiles/ckpt_mi355x.json
"""
from __future__ import annotations

import argparse
import json
import time
from typing import Dict, Sequence


def engine(device_index: int = 0, chunk_bytes: int = 1 << 30):
    import torch

    from ..ops import _lib

    _lib.load(required=True)
    return torch.classes.tam.CkptEngine(device_index, chunk_bytes)


def measure(device_index: int = 0, sizes_mb: Sequence[int] = (64, 256, 1024, 4096), reps: int = 3) -> Dict:
    import torch

    dev = torch.device("cuda", device_index)
    eng = engine(device_index, 1 << 30)
    rows = []
    for mb in sizes_mb:
        n = mb * (1 << 20) // 4
        x = torch.randn(n, device=dev)
        ref = x.clone()
        d2h, h2d = [], []
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            h = eng.spill(x)
            eng.wait(h)
            t1 = time.perf_counter()
            x.zero_()
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter()
            eng.restore(h, x)
            torch.cuda.synchronize(dev)
            t3 = time.perf_counter()
            eng.release(h)
            d2h.append(t1 - t0)
            h2d.append(t3 - t2)
        assert torch.equal(x, ref), "spill/restore round trip corrupted data"
        b = n * 4
        rows.append({"mb": mb, "d2h_gbps": round(b / min(d2h) / 1e9, 2),
                     "h2d_gbps": round(b / min(h2d) / 1e9, 2)})
        del x, ref
    p2p = None
    if torch.cuda.device_count() > 1:
        a = torch.empty(1 << 28, dtype=torch.uint8, device=dev)
        bdev = torch.device("cuda", (device_index + 1) % torch.cuda.device_count())
        bb = torch.empty_like(a, device=bdev)
        bb.copy_(a)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            bb.copy_(a)
        torch.cuda.synchronize()
        p2p = round(a.numel() * reps / (time.perf_counter() - t0) / 1e9, 2)
    big = rows[-1]
    return {"device": torch.cuda.get_device_name(dev), "engine_stats": list(eng.stats()),
            "d2h_gbps": big["d2h_gbps"], "h2d_gbps": big["h2d_gbps"], "p2p_gbps": p2p, "sweep": rows}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--out", default="profiles/ckpt_mi355x.json")
    a = ap.parse_args(argv)
    r = measure(a.device)
    print(json.dumps(r, indent=1))
    with open(a.out, "w") as f:
        json.dump(r, f, indent=1)


if __name__ == "__main__":
    main()
