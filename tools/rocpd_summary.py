"""Summarise a rocprofv3 rocpd database (ROCm 7 default output, run_results.db): per-kernel
count / total / average duration, like `--stats`, plus the wall span of the dispatches.

Usage: python tools/rocpd_summary.py DB [--top 25] [--csv OUT] [--match SUBSTR]
"""
import argparse
import csv
import sqlite3
from collections import defaultdict


def load(db, match=None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, stream_id, queue_id from kernels order by start").fetchall()
    if match:
        rows = [r for r in rows if match in r[0]]
    return rows


def stats(rows):
    agg = defaultdict(lambda: [0, 0])
    for name, s, e, *_ in rows:
        a = agg[name]
        a[0] += 1
        a[1] += e - s
    return sorted(((n, c, t) for n, (c, t) in agg.items()), key=lambda x: -x[2])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--csv")
    ap.add_argument("--match")
    a = ap.parse_args()
    rows = load(a.db, a.match)
    st = stats(rows)
    total = sum(t for _, _, t in st)
    span = (rows[-1][2] - rows[0][1]) if rows else 0
    print(f"{len(rows)} dispatches, kernel time {total / 1e6:.3f} ms, span {span / 1e6:.3f} ms, "
          f"streams {len(set(r[3] for r in rows))}, queues {len(set(r[4] for r in rows))}")
    for n, c, t in st[:a.top]:
        print(f"{t / 1e6:9.3f} ms {100 * t / max(total, 1):5.1f}% {c:7d} x {t / c / 1e3:9.2f} us  {n[:110]}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for n, c, t in st:
                w.writerow([n, c, t, t / c, 100 * t / max(total, 1)])


if __name__ == "__main__":
    main()
