#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (``-d DIR -o run`` -> DIR/run_results.db) as a
kernel-stats CSV: name, calls, total/avg/median/min/max in microseconds, share of GPU time.
``--skip-first N`` drops each kernel's first N dispatches (e.g. arena prefill / warmup)."""
import argparse
import csv
import sqlite3
import statistics
import sys
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--out", default="-")
    p.add_argument("--skip-first", type=int, default=0)
    p.add_argument("--top", type=int, default=30)
    a = p.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    d = defaultdict(list)
    for name, s, e in rows:
        d[name].append((e - s) / 1e3)
    for k in d:
        d[k] = d[k][a.skip_first:]
    tot = sum(sum(v) for v in d.values()) or 1.0
    out = sys.stdout if a.out == "-" else open(a.out, "w", newline="")
    w = csv.writer(out)
    w.writerow(["name", "calls", "total_us", "avg_us", "median_us", "min_us", "max_us", "pct"])
    for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[: a.top]:
        if not v:
            continue
        w.writerow([name[:160], len(v), round(sum(v), 1), round(sum(v) / len(v), 2), round(statistics.median(v), 2),
                    round(min(v), 2), round(max(v), 2), round(100 * sum(v) / tot, 2)])


if __name__ == "__main__":
    main()
