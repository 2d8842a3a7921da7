#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc counter CSVs (one row per dispatch x counter): MFMA busy,
achieved bf16 MFMA TFLOP/s and LDS bank-conflict rate, averaged over each kernel's dispatches.
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); TFLOP =
SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 per dispatch; conflict rate = SQ_LDS_BANK_CONFLICT /
SQ_LDS_IDX_ACTIVE."""
import csv
import re
import sys
from collections import defaultdict


def load(path):
    per = defaultdict(dict)
    names, dur = {}, {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
        dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return per, names, dur


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)[:48]


def main():
    mfma, lds = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None
    per, names, dur = load(mfma)
    agg = defaultdict(lambda: defaultdict(list))
    for d, c in per.items():
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in c or c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) == 0:
            continue
        k = short(names[d])
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        agg[k]["busy"].append(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024))
        agg[k]["tflop"].append(c["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / 1e12)
        agg[k]["us"].append(dur[d])
        agg[k]["ghz"].append(cyc / (dur[d] * 1e3))
    if lds:
        per2, names2, _ = load(lds)
        for d, c in per2.items():
            k = short(names2[d])
            if k in agg and c.get("SQ_LDS_IDX_ACTIVE", 0) > 0:
                agg[k]["conf"].append(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"])
    print("| kernel | dispatches | µs (profiled) | MFMA busy | TFLOP/s (MFMA ops / time) | GUI-active clock GHz | LDS conflict rate |")
    print("|---|---|---|---|---|---|---|")
    mean = lambda v: sum(v) / len(v) if v else float("nan")  # noqa: E731
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]["us"])):
        tf = mean([t / (u * 1e-6) for t, u in zip(v["tflop"], v["us"])])
        print(f"| `{k}` | {len(v['us'])} | {mean(v['us']):.1f} | {100 * mean(v['busy']):.1f} % | {tf:.0f} | "
              f"{mean(v['ghz']):.2f} | {100 * mean(v['conf']):.1f} % |")


if __name__ == "__main__":
    main()
