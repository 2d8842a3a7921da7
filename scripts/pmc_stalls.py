#!/usr/bin/env python3
"""Where each kernel's wave cycles go, from a rocprofv3 --pmc CSV with the SQ stall counters
(SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_LDS,
SQ_ACTIVE_INST_VALU, SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE).

WAIT_ANY (parked on s_waitcnt / barrier) + WAIT_INST_ANY (issue stalls) + ACTIVE_INST_ANY ~= WAVE_CYCLES
(MI355X_MICROARCH.md, rocprofv3 PMC slots).  MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8
XCDs x 1024 SIMDs).

python scripts/pmc_stalls.py COUNTER_COLLECTION.csv [--md] [--max-grid THREADS]

--max-grid: only dispatches of at most THREADS work-items (e.g. a KV step's slices and fused grid,
not the 2048-workgroup prepopulation inserts).
"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)[:48]


def main():
    path = sys.argv[1]
    per = defaultdict(dict)
    names, dur = {}, {}
    max_grid = int(sys.argv[sys.argv.index("--max-grid") + 1]) if "--max-grid" in sys.argv else 0
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        if max_grid:
            g = r.get("Grid_Size") or r.get("Grid_Size_X") or "0"
            if int(g) > max_grid:
                continue
        per[d][r["Counter_Name"]] = float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
        dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg = defaultdict(lambda: defaultdict(float))
    for d, c in per.items():
        if not c.get("SQ_WAVE_CYCLES"):
            continue
        k = short(names[d])
        for n, v in c.items():
            agg[k][n] += v
        agg[k]["_us"] += dur[d]
        agg[k]["_n"] += 1
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["_us"])
    print("| kernel | dispatches | µs avg | MFMA busy | wait (vmcnt/lgkm/barrier) | issue stall | of it LDS | active | active VALU |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k, c in rows:
        w = c["SQ_WAVE_CYCLES"]
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (c.get("GRBM_GUI_ACTIVE", 1) / 8 * 1024)
        f = lambda n: c.get(n, 0) / w * 100  # noqa: E731
        print(f"| `{k}` | {int(c['_n'])} | {c['_us'] / c['_n']:.1f} | {busy * 100:.1f} % | {f('SQ_WAIT_ANY'):.1f} % | "
              f"{f('SQ_WAIT_INST_ANY'):.1f} % | {f('SQ_WAIT_INST_LDS'):.1f} % | {f('SQ_ACTIVE_INST_ANY'):.1f} % | "
              f"{f('SQ_ACTIVE_INST_VALU'):.1f} % |")
    if "--md" not in sys.argv:
        return


if __name__ == "__main__":
    main()
