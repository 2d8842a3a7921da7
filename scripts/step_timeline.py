#!/usr/bin/env python3
"""Per-step phase breakdown of a bench.py kernel trace (rocprofv3 --kernel-trace rocpd db):
the KV phase (seqlock batch kernels) and the embed phase (encoder kernels) of each of the last
N steps, their spans, busy time and the gaps between kernels."""
import argparse
import sqlite3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--steps", type=int, default=5)
    a = p.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    kv = lambda n: "carry" in n or "rounds" in n or "k_set" in n or "k_get" in n  # noqa: E731
    # a step starts with a KV kernel that follows an encoder kernel
    steps, cur, prev_kv = [], [], False
    for n, s, e in rows:
        isk = kv(n)
        if isk and not prev_kv and cur:
            steps.append(cur)
            cur = []
        cur.append((n, s, e, isk))
        prev_kv = isk
    steps.append(cur)
    for st in steps[-a.steps:]:
        k = [r for r in st if r[3]]
        m = [r for r in st if not r[3]]
        t0 = st[0][1]
        ks = (max(r[2] for r in k) - min(r[1] for r in k)) / 1e3 if k else 0
        ms = (max(r[2] for r in m) - min(r[1] for r in m)) / 1e3 if m else 0
        mb = sum(r[2] - r[1] for r in m) / 1e3
        print(f"step: total {(max(r[2] for r in st) - t0) / 1e3:8.1f} us | KV span {ks:8.1f} us ({len(k)} kernels)"
              f" | embed span {ms:8.1f} us busy {mb:8.1f} us ({len(m)} kernels)")


if __name__ == "__main__":
    main()
