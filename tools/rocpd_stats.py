"""Per-kernel totals from a rocprofv3 SQLite output (rocpd `kernels` view):
name, calls, total / average ns, share -- the same columns as the
`--stats` kernel_stats.csv, for runs that wrote only the database.

  python tools/rocpd_stats.py gpurun_out/prof_rn/rn_results.db [--csv out.csv] [--top 25]
"""
import argparse
import csv
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default=None)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels "
                     f"group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    out = [{"Name": r[0], "Calls": r[1], "TotalDurationNs": int(r[2]), "AverageNs": round(r[3], 1),
            "Percentage": round(100.0 * r[2] / tot, 3)} for r in rows]
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)
    for r in out[:a.top]:
        print(f"{r['Percentage']:5.1f}% {r['Calls']:6d} {r['AverageNs'] / 1e3:8.1f}us {r['Name'][:100]}")
    print(f"total {tot / 1e6:.3f} ms over {sum(r['Calls'] for r in out)} dispatches", file=sys.stderr)


if __name__ == "__main__":
    main()
