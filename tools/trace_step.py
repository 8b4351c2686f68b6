"""Per-call view of ONE training step from a rocprofv3 kernel trace CSV:
the last occurrence of the step's first kernel (default: the ResNet stem)
to the end, with each call's duration, grid and the idle gap before it;
then totals per kernel family.

  python tools/trace_step.py gpurun_out/rn50_trace/run_kernel_trace.csv [--first conv_stem_fwd] [--rows]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(n):
    n = re.sub(r"\(.*", "", n)
    n = n.replace("void ", "").replace("tam::", "")
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--first", default="conv_stem_fwd")
    ap.add_argument("--rows", action="store_true")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.first in r["Kernel_Name"]]
    i0 = starts[-2] if len(starts) > 1 else starts[-1]
    i1 = starts[-1]
    step = rows[i0:i1]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = int(step[-1]["End_Timestamp"])
    fam = defaultdict(lambda: [0, 0.0, 0.0])
    prev_end = None
    busy = 0.0
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        d = (e - s) / 1e3
        busy += d
        k = short(r["Kernel_Name"])
        f = fam[k]
        f[0] += 1; f[1] += d; f[2] += max(gap, 0.0)
        if a.rows:
            print(f"{(s - t0) / 1e3:9.1f} {d:8.2f} gap {gap:6.2f} grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']} {k}")
        prev_end = max(prev_end or 0, e)
    span = (t1 - t0) / 1e3
    print(f"step span {span:.1f} us, kernels {len(step)}, busy {busy:.1f} us, idle {span - busy:.1f} us")
    for k, (n, d, g) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"{d:9.1f} us {100 * d / span:5.1f}% n={n:4d} avg {d / n:7.2f} gaps {g:7.1f}  {k}")


if __name__ == "__main__":
    main()
