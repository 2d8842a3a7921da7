#!/bin/bash
# search pass with the conflict-free row swizzle for gfx950's ds_read_b128 lane groups: search tests,
# interleaved A/B against the previous commit (libsplinter_hip_prev.so), LDS conflict rate
set -o pipefail
OUT=gpurun_out/r5swz
mkdir -p $OUT
ROOT=$(pwd)
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/search_tests.txt 2>&1 || { tail -30 $OUT/search_tests.txt; exit 1; }
tail -1 $OUT/search_tests.txt
for r in 1 2; do
  for v in new prev; do
    if [ $v = new ]; then unset SPLINTER_HIP_VARIANT; else export SPLINTER_HIP_VARIANT=$v; fi
    timeout -k 10 400 python3 scripts/search_bench.py --nq 256 --iters 3 > $OUT/$v$r.out 2> $OUT/$v$r.err || { tail -20 $OUT/$v$r.err; exit 1; }
    echo "$v $r: $(python3 -c "import json; d=json.loads(open('$OUT/$v$r.out').read().strip().splitlines()[-1]); print(round(d['qps']), d['recall_at_k'], d['exact_match'], round(d['ms_per_batch'],2))")"
  done
done
unset SPLINTER_HIP_VARIANT
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d "$ROOT/$OUT/pmc" -o run -- python3 scripts/search_bench.py --nq 256 --iters 2 > $OUT/pmc.out 2> $OUT/pmc.err || { tail -20 $OUT/pmc.err; exit 1; }
csv=$(find "$OUT/pmc" -name '*counter_collection.csv' | head -1)
python3 - "$csv" <<'PY'
import csv, sys, collections
d = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_search_mma16<1>" in r["Kernel_Name"]:
        d[r["Counter_Name"]] += float(r["Counter_Value"])
print({k: round(v) for k, v in d.items()}, "conflict rate", round(d["SQ_LDS_BANK_CONFLICT"] / max(d["SQ_LDS_IDX_ACTIVE"], 1), 3))
PY
rm -rf $OUT/pmc
