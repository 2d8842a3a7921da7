#!/bin/bash
# timed-region kernel trace of the final tree's mixed step (scripts/trace_window.py)
set -o pipefail
OUT=gpurun_out/r5trace
mkdir -p $OUT
ROOT=$(pwd)
export TMPDIR=/tmp
SPL_PROFILE_TIMED=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/tr" -o run \
  -- python3 bench.py --steps 10 --warmup 3 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 \
  --exchange-ab 0 --mixed5 0 --search-keys 0 > $OUT/native.out 2> $OUT/native.err || { tail -20 $OUT/native.err; exit 1; }
csv=$(find "$OUT/tr" -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_window.py "$csv" "$OUT/native.err" --md "$OUT/trace_native.md" --timeline || exit 1
rm -rf "$OUT/tr"
head -30 "$OUT/trace_native.md"
