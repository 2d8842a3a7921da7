#!/bin/bash
# Search (config #5) on one MI355X: the search GPU tests, scripts/search_bench.py at 25 M slots
# (512-query batches), and a kernel-trace summary of it.  Each step has its own limit.
set -o pipefail
OUT=${OUT:-gpurun_out/search}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_search_gpu.py -m gpu -x -v --timeout 150 --timeout-method thread \
  > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
timeout -k 10 300 python -u scripts/search_bench.py --slots 25000000 --nq 512 --iters 3 > "$OUT/bench.out" 2> "$OUT/bench.err" \
  || { tail -20 "$OUT/bench.err"; exit 1; }
tail -3 "$OUT/bench.out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" \
  -o run -- python -u scripts/search_bench.py --slots 25000000 --nq 512 --iters 2 > "$OUT/prof.out" 2>&1 \
  || { tail -20 "$OUT/prof.out"; exit 1; }
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
if [ -n "$f" ]; then head -12 "$f"; fi
if [ -n "$PMC" ]; then  # SQ wave-cycle split of the search kernels (one pass, its own run)
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES \
    GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc" -o run -- python3 scripts/search_bench.py --slots 25000000 \
    --nq 512 --iters 1 > "$OUT/pmc.out" 2>&1 || { tail -20 "$OUT/pmc.out"; exit 1; }
  csv=$(find "$OUT/pmc" -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_stalls.py "$csv" --md --max-grid 1000000 > "$OUT/pmc.md" || exit 1
  cat "$OUT/pmc.md"; gzip -f "$csv"
fi
exit 0
