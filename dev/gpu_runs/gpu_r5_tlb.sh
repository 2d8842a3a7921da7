#!/bin/bash
# fused KV grid (bench.py --mode kv, 100 M keys): address-translation and L2 / DRAM request counters
set -o pipefail
OUT=gpurun_out/r5tlb
mkdir -p $OUT
ROOT=$(pwd)
export TMPDIR=/tmp
i=0
for ctr in "TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $ctr --output-format csv -d "$ROOT/$OUT/p$i" -o run -- python3 bench.py --mode kv \
    --steps 3 --warmup 1 --host-api 0 --host-api-threads2 0 --exchange-ab 0 > "$OUT/kv$i.out" 2> "$OUT/kv$i.err" || { tail -20 "$OUT/kv$i.err"; exit 1; }
  csv=$(find "$OUT/p$i" -name '*counter_collection.csv' | head -1)
  python3 - "$csv" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0][-60:]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    if "kv_fused" in k or "set_carry" in k or "get_carry" in k:
        print(k, {c: (v, n[(k, c)]) for c, v in d.items()})
PY
  gzip -f "$csv"
done
