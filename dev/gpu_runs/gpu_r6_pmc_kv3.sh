#!/bin/bash
# KV-only fused grid PMC, get output rows exact (0) vs through whole 64-B lines (1, default): SQ split and
# split and the L2 / memory requests per op (16 M ops per dispatch)
set -o pipefail
OUT=gpurun_out/r6pmckv3
mkdir -p $OUT
ROOT=$(pwd)
export TMPDIR=/tmp
ARGS="--mode kv --steps 4 --warmup 2 --host-api 0 --host-api-threads2 0 --exchange-ab 0 --kv-async-ab 0"
for s in 0 1; do
  SPL_KVS_PAD_OUT=$s timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$ROOT/$OUT/sq$s" -o run -- python3 bench.py $ARGS > "$OUT/sq$s.out" 2> "$OUT/sq$s.err" || { tail -20 "$OUT/sq$s.err"; exit 1; }
  csv=$(find "$OUT/sq$s" -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_stalls.py "$csv" --md --max-grid 200000 > "$OUT/sq$s.md" || exit 1
  echo "== pad_out $s SQ"; grep k_kv_fused "$OUT/sq$s.md"
  rm -f "$csv"
  SPL_KVS_PAD_OUT=$s timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum \
    GRBM_GUI_ACTIVE --output-format csv -d "$ROOT/$OUT/tcc$s" -o run -- python3 bench.py $ARGS > "$OUT/tcc$s.out" 2> "$OUT/tcc$s.err" || { tail -20 "$OUT/tcc$s.err"; exit 1; }
  csv=$(find "$OUT/tcc$s" -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_req_summary.py "$csv" k_kv_fused 16000000 > "$OUT/tcc$s.md" || exit 1
  echo "== pad_out $s TCC"; cat "$OUT/tcc$s.md"
  rm -f "$csv"
done
