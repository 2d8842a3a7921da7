#!/bin/bash
# SQ wave-cycle split (parked on waits / issue-stalled / active) of the KV step's kernels, per-slice
# dispatches (SPL_KVS_FUSED=0) vs the fused grid (2): bench.py --mode kv (100 M keys, 32+32 streams).
# Counter collection serialises dispatches, so the per-dispatch times are single-dispatch times.
set -o pipefail
OUT=${OUT:-gpurun_out/pmc_kv}
mkdir -p "$OUT"
ROOT=$(pwd)
export TMPDIR=/tmp
for f in 0 2; do
  SPL_KVS_FUSED=$f timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$ROOT/$OUT/pmc_kv$f" -o run -- python3 bench.py --mode kv \
    --steps 5 --warmup 2 --host-api 0 --host-api-threads2 0 --exchange-ab 0 > "$OUT/kv$f.out" 2> "$OUT/kv$f.err"
  rc=$?
  echo "== kv$f rc=$rc"; tail -c 400 "$OUT/kv$f.out"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/kv$f.err"; exit $rc; fi
  csv=$(find "$OUT/pmc_kv$f" -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_stalls.py "$csv" --md --max-grid 200000 > "$OUT/pmc_kv$f.md" || exit 1
  cat "$OUT/pmc_kv$f.md"
  gzip -f "$csv"
done
exit 0
