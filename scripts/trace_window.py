#!/usr/bin/env python3
"""Cut a rocprofv3 kernel trace (CSV, ``--kernel-trace --output-format csv``) to the timed region of
a ``SPL_PROFILE_TIMED=1`` bench.py run and summarise it per kernel.

python scripts/trace_window.py KERNEL_TRACE.csv BENCH_STDERR.log [--md OUT.md] [--csv OUT.csv]

bench.py prints the region's bounds in the monotonic and the boot-time clock; the clock whose
window holds kernel dispatches is used.  Vendor-library and framework kernels (hipBLASLt ``Cijk_``,
rocBLAS, ``at::native``) inside the window are listed separately: the timed step should have none.
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("log")
    ap.add_argument("--md")
    ap.add_argument("--csv")
    ap.add_argument("--timeline", action="store_true",
                    help="also the wall time each kernel (and all of them) is running: the union of its dispatch "
                         "intervals, which shows which of concurrently running kernel groups bounds the region")
    a = ap.parse_args()
    bounds = {}
    for line in open(a.log, errors="replace"):
        line = line.strip()
        if line.startswith("{") and "timed_region" in line:
            d = json.loads(line)
            bounds[d["timed_region"]] = d
    rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(a.trace))]
    best = None
    for clk in ("monotonic_ns", "boottime_ns"):
        lo, hi = bounds["begin"][clk], bounds["end"][clk]
        inside = [r for r in rows if lo <= r[1] and r[2] <= hi]
        if best is None or len(inside) > len(best[1]):
            best = (clk, inside, hi - lo)
    clk, inside, span = best
    agg = defaultdict(list)
    for n, s, e in inside:
        agg[n].append((e - s) / 1e3)
    tot = sum(sum(v) for v in agg.values()) or 1.0
    vendor = [n for n in agg if re.search(r"Cijk_|rocblas|at::native|hipblaslt|Tensile", n)]
    lines = [f"timed region: {span / 1e6:.2f} ms ({clk}); {len(inside)} kernel dispatches, "
             f"{tot / 1e3:.2f} ms of kernel time; vendor/framework kernels inside: {len(vendor)}", "",
             "| kernel | calls | total ms | avg us | share |", "|---|---|---|---|---|"]
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| `{short(n)}` | {len(v)} | {sum(v) / 1e3:.3f} | {sum(v) / len(v):.1f} | {sum(v) / tot * 100:.1f} % |")
    if vendor:
        lines += ["", "vendor / framework kernels in the timed region:"] + [f"- `{short(n)}`" for n in vendor]
    if a.timeline:
        def union(iv):
            tot, end = 0, None
            for s0, e0 in sorted(iv):
                if end is None or s0 > end:
                    tot += e0 - s0
                    end = e0
                elif e0 > end:
                    tot += e0 - end
                    end = e0
            return tot
        groups = defaultdict(list)
        for n, s0, e0 in inside:
            groups[short(n)].append((s0, e0))
        lines += ["", "| kernel | wall time running (union of dispatches) ms | share of region |", "|---|---|---|"]
        for n, iv in sorted(groups.items(), key=lambda kv: -union(kv[1])):
            lines.append(f"| `{n}` | {union(iv) / 1e6:.3f} | {union(iv) / span * 100:.1f} % |")
        allv = [(s0, e0) for _, s0, e0 in inside]
        lines.append(f"| any kernel | {union(allv) / 1e6:.3f} | {union(allv) / span * 100:.1f} % |")
    out = "\n".join(lines)
    print(out)
    if a.md:
        open(a.md, "w").write(out + "\n")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["name", "calls", "total_us", "avg_us", "pct"])
            for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
                w.writerow([n, len(v), round(sum(v), 1), round(sum(v) / len(v), 2), round(sum(v) / tot * 100, 2)])


if __name__ == "__main__":
    main()
