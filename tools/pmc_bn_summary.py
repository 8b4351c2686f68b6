"""Per-dispatch HBM traffic of the BatchNorm kernels from two rocprofv3 PMC
passes (FETCH_SIZE, WRITE_SIZE; kilobytes per dispatch): dispatches are
joined by their order within each kernel name, and bytes / duration gives
the achieved HBM rate. Prints per kernel name the aggregate rate and the
rates of its largest dispatches."""
import glob
import sqlite3
import sys
from collections import defaultdict


def load(d, counter):
    db = sorted(glob.glob(f"{d}/{counter}/**/*.db", recursive=True))[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, dispatch_id, duration, counter_name, counter_value from pmc_events").fetchall()
    per = defaultdict(dict)
    for name, disp, dur, cn, cv in rows:
        if not name.startswith("bn_") and "bn_" not in name:
            continue
        e = per[name].setdefault(disp, [float(dur), 0.0])
        e[1] += float(cv)
    return {n: [v for _, v in sorted(d.items())] for n, d in per.items()}


def main():
    d = sys.argv[1]
    f, w = load(d, "FETCH_SIZE"), load(d, "WRITE_SIZE")
    for name in sorted(f):
        rows = []
        for (dur_ns, kb_r), (_, kb_w) in zip(f[name], w.get(name, [])):
            rows.append((dur_ns / 1e3, kb_r * 1024, kb_w * 1024))
        if not rows:
            continue
        tot_us = sum(r[0] for r in rows)
        tot_b = sum(r[1] + r[2] for r in rows)
        big = sorted(rows, key=lambda r: -(r[1] + r[2]))[:5]
        print(f"{name[:40]:40s} n={len(rows):4d} time {tot_us:9.1f} us  bytes {tot_b / 1e9:7.2f} GB  "
              f"rate {tot_b / tot_us / 1e6:5.2f} TB/s")
        for us, r, wb in big:
            print(f"    {us:7.1f} us  read {r / 1e6:7.1f} MB  write {wb / 1e6:7.1f} MB  {(r + wb) / us / 1e6:5.2f} TB/s")


if __name__ == "__main__":
    main()
