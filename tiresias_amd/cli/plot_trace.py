"""Trace sanity plots / statistics (the reference's ``demonstrate_trace.py``
plots the synthetic generator's CDFs with matplotlib). matplotlib is not
installed here, so this prints the CDF quantiles as text and writes them to
CSV; if matplotlib is importable it also saves PNGs.

    python -m tiresias_amd.cli.plot_trace --synthetic 1000 --out log/trace_cdf
    python -m tiresias_amd.cli.plot_trace --trace_file trace.csv
"""
from __future__ import annotations

import argparse
import csv
import os

from ..trace import readers, synth

QS = [0.01, 0.1, 0.25, 0.5, 0.75, 0.9, 0.99]


def quantiles(xs, qs=QS):
    s = sorted(xs)
    return [s[min(len(s) - 1, int(q * (len(s) - 1)))] for q in qs] if s else [0] * len(qs)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace_file", default="")
    ap.add_argument("--synthetic", type=int, default=0)
    ap.add_argument("--sample_generator", action="store_true", help="use the reference sample populations")
    ap.add_argument("--gpus", type=int, default=64)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    if a.trace_file:
        specs = readers.read_trace(a.trace_file)
    elif a.sample_generator:
        specs = synth.SampleTraceGenerator(a.seed).generate_specs(a.synthetic or 1000)
    else:
        specs = synth.philly_like_trace(a.synthetic or 1000, a.gpus, seed=a.seed)
    assert specs, "empty trace"
    cols = {
        "duration": [s.duration for s in specs],
        "num_gpu": [s.num_gpu for s in specs],
        "gpu_service": [s.duration * s.num_gpu for s in specs],
        "interarrival": [b.submit_time - a_.submit_time for a_, b in zip(specs, specs[1:])] or [0],
    }
    print(f"{'metric':14s} " + " ".join(f"p{int(q * 100):02d}".rjust(10) for q in QS))
    rows = []
    for k, v in cols.items():
        qv = quantiles(v)
        rows.append([k] + qv)
        print(f"{k:14s} " + " ".join(f"{x:10.2f}" for x in qv))
    if a.out:
        os.makedirs(a.out, exist_ok=True)
        with open(os.path.join(a.out, "cdf.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["metric"] + [f"p{int(q * 100)}" for q in QS])
            w.writerows(rows)
        try:
            import matplotlib

            matplotlib.use("Agg")
            import matplotlib.pyplot as plt

            for k, v in cols.items():
                s = sorted(v)
                plt.figure()
                plt.plot(s, [i / max(1, len(s) - 1) for i in range(len(s))])
                plt.xlabel(k)
                plt.ylabel("CDF")
                plt.savefig(os.path.join(a.out, f"{k}_cdf.png"))
                plt.close()
        except ImportError:
            pass
    return rows


if __name__ == "__main__":
    main()
