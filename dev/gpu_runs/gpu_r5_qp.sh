#!/bin/bash
# timing probe: two-wave search pass with the query fragments read from LDS once per tile (wrong
# results) vs every step: LDS conflict rate and pass time
set -o pipefail
OUT=gpurun_out/r5qp
mkdir -p $OUT
ROOT=$(pwd)
export TMPDIR=/tmp
for v in base qprobe; do
  if [ $v = base ]; then unset SPLINTER_HIP_VARIANT; else export SPLINTER_HIP_VARIANT=$v; fi
  timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d "$ROOT/$OUT/$v" -o run -- python3 scripts/search_bench.py --nq 256 --iters 2 > $OUT/$v.out 2> $OUT/$v.err || { tail -20 $OUT/$v.err; exit 1; }
  csv=$(find "$OUT/$v" -name '*counter_collection.csv' | head -1)
  python3 - "$csv" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "k_search_mma16<1>" in r["Kernel_Name"]:
        agg["p1"][r["Counter_Name"]] += float(r["Counter_Value"])
        agg["p1"]["_dur"] += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3 / 5
d = agg["p1"]
print({k: round(v) for k, v in d.items()}, "conflict", round(d["SQ_LDS_BANK_CONFLICT"] / max(d["SQ_LDS_IDX_ACTIVE"], 1), 3))
PY
  rm -rf $OUT/$v
done
