#!/bin/bash
# PMC of the two-wave search pass (search_bench, 256 queries over 25 M x 768): MFMA busy, LDS, stalls
set -o pipefail
OUT=gpurun_out/r5spmc
mkdir -p $OUT
ROOT=$(pwd)
export TMPDIR=/tmp
run() {  # run NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --output-format csv -d "$ROOT/$OUT/$name" -o run -- python3 scripts/search_bench.py \
    --nq 256 --iters 2 > "$OUT/$name.out" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  find "$OUT/$name" -name '*counter_collection.csv' | head -1
}
m=$(run mfma SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE) || exit 1
l=$(run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE) || exit 1
w=$(run stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE) || exit 1
python3 scripts/pmc_summary.py "$m" "$l" > "$OUT/pmc_search.md" || exit 1
python3 scripts/pmc_stalls.py "$w" --md --max-grid 200000 > "$OUT/stall_search.md" || exit 1
cat "$OUT/pmc_search.md" "$OUT/stall_search.md" | grep -i "search\|rescore\|kernel |"
gzip -f "$m" "$l" "$w"
