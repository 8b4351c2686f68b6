"""ResNet-50 stem forward (7x7 / s2 / p3, 8 -> 64 channels, batch 64 at
224x224, with the BatchNorm sums): the dedicated kernel (conv_stem.hip) vs
the generic conv paths, interleaved, best of 5 bursts of 20.

  python tools/bench_stem.py [--batch 64]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402
from tiresias_amd.ops.functional import BN_SHARDS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    _lib.load(required=True)
    T = torch.ops.tam
    dev = torch.device("cuda", 0)
    x = torch.randn(a.batch, 224, 224, 8, device=dev).to(torch.bfloat16)
    w = (torch.randn(64, 7, 7, 8, device=dev) / 20).to(torch.bfloat16)
    y = torch.empty(a.batch, 112, 112, 64, device=dev, dtype=torch.bfloat16)
    sums = torch.zeros(BN_SHARDS * 128, device=dev, dtype=torch.float64)
    run = lambda: T.conv_fwd(x, w, y, 2, 3, 1, None, False, sums)  # noqa: E731
    dy = torch.randn(a.batch, 112, 112, 64, device=dev).to(torch.bfloat16)
    dw = torch.zeros(64, 7, 7, 8, device=dev)
    runw = lambda: T.conv_wgrad(dy, x, dw, 2, 3, 1, 1)  # noqa: E731
    best = {}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        for pol in (1, 0):
            T.conv_stem_policy(pol)
            for _ in range(3):
                run()
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            torch.cuda.synchronize()
            best[pol] = min(best.get(pol, 1e9), e0.elapsed_time(e1) / 20 * 1e3)
            for _ in range(3):
                runw()
            e0.record()
            for _ in range(20):
                runw()
            e1.record()
            torch.cuda.synchronize()
            best[pol + 2] = min(best.get(pol + 2, 1e9), e0.elapsed_time(e1) / 20 * 1e3)
    T.conv_stem_policy(1)
    fl = 2.0 * a.batch * 112 * 112 * 64 * 392
    print(json.dumps({"batch": a.batch, "stem_us": round(best[1], 2), "generic_us": round(best[0], 2),
                      "stem_tflops": round(fl / best[1] / 1e6, 1), "generic_tflops": round(fl / best[0] / 1e6, 1),
                      "wgrad_stem_us": round(best[3], 2), "wgrad_generic_us": round(best[2], 2)}))


if __name__ == "__main__":
    main()
