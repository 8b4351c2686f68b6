"""Do two independent persistent LSTM recurrences gain from running at once?

GNMT has two pairs of recurrences with no data dependence between them (the
two directions of the bidirectional encoder layer; the first decoder layer
and the encoder stack). Each persistent grid is 256 workgroups (one per CU)
and its per-timestep cost is hand-off latency, so a second grid co-resident
on the same CUs (two workgroups per CU fit) could overlap almost for free.
This times, per pass (forward / backward, GNMT shapes T=50, B=64, H=1024):

  one   : one launch
  seq   : two launches on one stream
  pair  : two launches on two streams, issued together

    python tools/bench_lstm_pair.py [--one]   (--one: 10 single launches, for PMC)
"""
from __future__ import annotations

import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

BF = torch.bfloat16


def main():
    _lib.load(required=True)
    T_ops = torch.ops.tam
    dev = torch.device("cuda", 0)
    T, B, H = 50, 64, 1024
    torch.manual_seed(0)

    def make():
        return dict(gx=torch.randn(T, B, 4 * H, device=dev),
                    w=(torch.randn(4 * H, H, device=dev) / H ** 0.5).to(BF),
                    hs=torch.empty(T, B, H, device=dev, dtype=BF),
                    cs=torch.empty(T, B, H, device=dev), act=torch.empty(T, B, 5 * H, device=dev),
                    dH=torch.randn(T, B, H, device=dev).to(BF),
                    dG=torch.empty(T, B, 4 * H, device=dev, dtype=BF),
                    sync=torch.zeros(32 * (4 * (B // 16) + 1), dtype=torch.int32, device=dev))

    js = [make(), make()]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]

    def fwd(j, rev):
        assert T_ops.lstm_seq_forward(j["gx"], j["w"], j["hs"], j["cs"], j["act"], rev, j["sync"])

    def bwd(j, rev):
        assert T_ops.lstm_seq_backward(j["act"], j["cs"], j["dH"], j["w"], j["dG"], rev, j["sync"])

    def timed(fn, iters=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(3):
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / iters * 1e3)
        return best

    def pair(op):
        def run():
            cur = torch.cuda.current_stream(dev)
            ev = torch.cuda.Event()
            ev.record(cur)
            for k in (0, 1):
                streams[k].wait_event(ev)
                with torch.cuda.stream(streams[k]):
                    op(js[k], k == 1)
            for k in (0, 1):
                cur.wait_stream(streams[k])
        return run

    if "--one" in sys.argv:                    # single launches only (PMC passes)
        for _ in range(10):
            fwd(js[0], False)
            bwd(js[0], False)
        torch.cuda.synchronize()
        return
    out = {}
    for name, op in (("fwd", fwd), ("bwd", bwd)):
        fwd(js[0], False)
        fwd(js[1], True)
        out[name] = dict(one_us=round(timed(lambda: op(js[0], False)), 1),
                         seq_us=round(timed(lambda: (op(js[0], False), op(js[1], True))), 1),
                         pair_us=round(timed(pair(op)), 1))
        torch.cuda.synchronize()
        out[name]["timeouts"] = int(js[0]["sync"][0]) + int(js[1]["sync"][0])
        print(name, json.dumps(out[name]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
