#!/bin/bash
# MFMA busy / TFLOP/s and LDS conflict rate of the encoder kernels (bench.py --mode embed, 64 x 512
# tokens, 12 layers) with the current defaults: one rocprofv3 --pmc pass per counter group, each
# its own run (counter collection serialises dispatches: the us column is single-dispatch time).
set -o pipefail
OUT=${OUT:-gpurun_out/pmc_enc}
mkdir -p "$OUT"
ROOT=$(pwd)
export TMPDIR=/tmp
run() {  # run NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --output-format csv -d "$ROOT/$OUT/$name" -o run -- python3 bench.py \
    --mode embed --steps 2 --warmup 1 > "$OUT/$name.out" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  find "$OUT/$name" -name '*counter_collection.csv' | head -1
}
m=$(run mfma SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE) || exit 1
l=$(run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE) || exit 1
python3 scripts/pmc_summary.py "$m" "$l" > "$OUT/pmc_encoder.md" || exit 1
cat "$OUT/pmc_encoder.md"
gzip -f "$m" "$l"
exit 0
