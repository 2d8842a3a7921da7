#!/usr/bin/env python3
"""Per-kernel mean of every counter in rocprofv3 --pmc result databases (ROCm 7.2 writes
run_results.db, SQLite): python scripts/pmc_db_summary.py DB [DB ...] [--filter SUBSTR].
Prints one line per (kernel, counter) plus derived MFMA busy / clock / wait shares when the
counters are present."""
import argparse
import collections
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for db in a.dbs:
        c = sqlite3.connect(db)
        rows = c.execute("select dispatch_id, kernel_name, counter_name, value, duration from counters_collection")
        seen = set()
        for d, k, n, v, dur in rows:
            k = re.sub(r"\(.*", "", k.replace("void ", "").replace("(anonymous namespace)::", ""))[:70]
            if a.filter and a.filter not in k:
                continue
            agg[k][n].append(float(v))
            if (db, d) not in seen:
                seen.add((db, d))
                agg[k]["_us"].append(dur / 1e3)
    for k, cs in agg.items():
        m = {n: sum(v) / len(v) for n, v in cs.items()}
        out = {n: (round(x, 3) if abs(x) < 1e4 else int(x)) for n, x in sorted(m.items())}
        if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            cyc = m["GRBM_GUI_ACTIVE"] / 8
            out["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024), 3)
            out["clock_ghz"] = round(cyc / (m["_us"] * 1e3), 3)
        if "SQ_WAVE_CYCLES" in m:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if n in m:
                    out[n + "_share"] = round(m[n] / m["SQ_WAVE_CYCLES"], 3)
        if "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
            out["lds_conflict_rate"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 4)
        print(k, len(cs["_us"]), out)


if __name__ == "__main__":
    main()
