#!/bin/bash
# Timed-region kernel traces of the native and the routed (--force-routed, world 1) mixed step:
# which kernels run in the measured steps and how long (scripts/trace_window.py).  One MI355X.
set -o pipefail
OUT=${OUT:-gpurun_out/trace_routed}
mkdir -p "$OUT"
ROOT=$(pwd)
export TMPDIR=/tmp
ARGS="--steps 10 --warmup 3 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0"
for mode in native routed; do
  extra=""; [ $mode = routed ] && extra="--force-routed"
  SPL_PROFILE_TIMED=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/tr_$mode" -o run \
    -- python3 bench.py $ARGS $extra > "$OUT/$mode.out" 2> "$OUT/$mode.err"
  rc=$?
  echo "== $mode rc=$rc"; tail -c 600 "$OUT/$mode.out"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$mode.err"; exit $rc; fi
  csv=$(find "$OUT/tr_$mode" -name '*kernel_trace.csv' | head -1)
  python3 scripts/trace_window.py "$csv" "$OUT/$mode.err" --md "$OUT/trace_$mode.md" --timeline || exit 1
  rm -f "$csv"
  head -25 "$OUT/trace_$mode.md"
done
exit 0
