#!/usr/bin/env python3
"""Memory requests per KV op of a kernel, from a rocprofv3 --pmc CSV with the TCC request counters
(TCC_EA0_RDREQ_sum / TCC_EA0_WRREQ_sum: L2 -> memory read / write requests, TCC_HIT_sum /
TCC_MISS_sum: L2 lookups) -- the per-op request budget of the fused KV grid.

python scripts/pmc_req_summary.py COUNTER_COLLECTION.csv KERNEL_SUBSTRING OPS_PER_DISPATCH
"""
import csv
import sys
from collections import defaultdict


def main():
    path, sub, ops = sys.argv[1], sys.argv[2], float(sys.argv[3])
    per = defaultdict(dict)
    dur = {}
    for r in csv.DictReader(open(path)):
        if sub not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if not per:
        print(f"no dispatch of {sub}")
        return 1
    n = len(per)
    tot = defaultdict(float)
    for c in per.values():
        for k, v in c.items():
            tot[k] += v / n
    us = sum(dur.values()) / n
    rd, wr = tot.get("TCC_EA0_RDREQ_sum", 0), tot.get("TCC_EA0_WRREQ_sum", 0)
    hit, miss = tot.get("TCC_HIT_sum", 0), tot.get("TCC_MISS_sum", 0)
    print("| dispatches | us avg | L2 lookups / op | L2 hit rate | memory reads / op | memory writes / op | memory requests / s |")
    print("|---|---|---|---|---|---|---|")
    look = hit + miss
    print(f"| {n} | {us:.1f} | {look / ops:.2f} | {hit / max(look, 1) * 100:.1f} % | {rd / ops:.2f} | {wr / ops:.2f} | "
          f"{(rd + wr) / (us * 1e-6) / 1e9:.1f} G |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
