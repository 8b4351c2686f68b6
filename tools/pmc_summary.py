"""Summarise rocprofv3 PMC .db files (one per pass): per kernel name,
the median over dispatches of each counter and of the duration."""
import glob
import sqlite3
import statistics
import sys
from collections import defaultdict


def summarize(db, match=""):
    c = sqlite3.connect(db)
    rows = c.execute("select name, dispatch_id, duration, counter_name, counter_value from pmc_events").fetchall()
    per = defaultdict(lambda: defaultdict(dict))
    for name, disp, dur, cn, cv in rows:
        if match and match not in name:
            continue
        per[name][disp][cn] = per[name][disp].get(cn, 0.0) + float(cv)
        per[name][disp]["_dur_us"] = float(dur) / 1e3
    out = {}
    for name, d in per.items():
        keys = set(k for v in d.values() for k in v)
        out[name] = {k: statistics.median(v.get(k, 0.0) for v in d.values()) for k in keys}
        out[name]["_n"] = len(d)
    return out


if __name__ == "__main__":
    match = sys.argv[2] if len(sys.argv) > 2 else ""
    for db in sorted(glob.glob(sys.argv[1] + "/**/*.db", recursive=True)):
        for k, v in summarize(db, match).items():
            print(db.split("/")[-2], k[:60], {a: round(b, 1) for a, b in sorted(v.items())})
