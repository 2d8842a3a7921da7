#!/bin/bash
# Node batch ABI on one MI355X (4 HBM shards on device 0): GPU batch tests, then
# splinter_hostapi_bench --batch on hbm: and node: at SPLINTER_NODE_BATCH_THREADS 8 / 16, one
# traced run (per-phase ms of every batch).  Each step has its own limit; any failure ends it.
set -o pipefail
OUT=${OUT:-gpurun_out/nb}
mkdir -p "$OUT"
H=./libsplinter_amd/bin/splinter_hostapi_bench
timeout -k 10 300 python -u -m pytest tests/test_batch_api.py -m gpu -x -v --timeout 150 --timeout-method thread \
  > "$OUT/tests.log" 2>&1 || { tail -20 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
timeout -k 10 120 $H --store hbm:nb0 --batch 2000000 --keys 8000000 --seconds 3 > "$OUT/hbm.out" 2> "$OUT/hbm.err" || exit 1
tail -1 "$OUT/hbm.out"
for t in ${THREADS:-8 16}; do
  for r in 1 2; do
    SPLINTER_NODE_SHARDS=4 SPLINTER_NODE_BATCH_THREADS=$t timeout -k 10 120 $H --store node:nb$t$r --batch 2000000 \
      --keys 8000000 --seconds 3 > "$OUT/node_t${t}_$r.out" 2> "$OUT/node_t${t}_$r.err" || exit 1
    echo "t$t r$r $(tail -1 $OUT/node_t${t}_$r.out)"
  done
done
SPLINTER_NODE_SHARDS=4 SPLINTER_NODE_BATCH_TRACE=1 timeout -k 10 120 $H --store node:nbtr --batch 2000000 --keys 8000000 \
  --seconds 3 > "$OUT/node_trace.out" 2> "$OUT/node_trace.err" || exit 1
tail -1 "$OUT/node_trace.out"; tail -4 "$OUT/node_trace.err"
